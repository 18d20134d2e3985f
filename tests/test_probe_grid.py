"""ProbeGrid.from_bounding_box = Scene::generateProbeGridFromBoundingBox
(arkose/scene/Scene.cpp:534-583): 1 m margin, 16 probes per axis, 32 on the largest
axis chosen by the reference's rule (:563-570), fp32 spacing and origin."""
import numpy as np
import pytest

from arkoserenderer_amd import ddgi as D


@pytest.mark.parametrize("lo,hi,largest", [
    ((0, 0, 0), (10, 4, 3), 0),   # x largest
    ((0, 0, 0), (3, 10, 4), 1),   # y largest
    ((0, 0, 0), (3, 4, 10), 2),   # z largest
    ((0, 0, 0), (3, 10, 10), 2),  # y == z > x: the reference picks z (y > z is false)
    ((0, 0, 0), (10, 10, 3), 0),  # x == y > z: neither y nor z exceeds x -> x
    ((0, 0, 0), (10, 3, 10), 0),  # x == z > y -> x
    ((0, 0, 0), (5, 5, 5), 0),    # all equal -> x
    ((-2, -1, -3), (2, 8, 5), 1),  # bounds (6, 11, 10): y
])
def test_largest_axis_rule(lo, hi, largest):
    g = D.ProbeGrid.from_bounding_box(lo, hi)
    want = [16, 16, 16]
    want[largest] = 32
    assert list(g.grid_dimensions) == want
    lo32 = np.asarray(lo, np.float32) - np.float32(1)
    hi32 = np.asarray(hi, np.float32) + np.float32(1)
    bounds = hi32 - lo32
    assert np.array_equal(np.asarray(g.offset_to_first, np.float32), lo32)
    assert np.array_equal(np.asarray(g.probe_spacing, np.float32), (bounds / np.asarray(want, np.float32)).astype(np.float32))


def test_grid_spans_the_grown_box():
    g = D.ProbeGrid.from_bounding_box((0.5, -1.25, 2.0), (7.5, 3.0, 9.0))
    last = np.asarray(g.offset_to_first) + np.asarray(g.probe_spacing) * np.asarray(g.grid_dimensions)
    assert np.allclose(last, np.asarray((8.5, 4.0, 10.0)), atol=1e-5)
