"""The oracle reproduces the committed golden fixtures bit for bit (sha256 per
frame and resource), and its fp16 rounding matches the reference's half.hpp."""
import hashlib
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden as G  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    f = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    return dict(zip(f["keys"].tolist(), f["values"].tolist())), f["last_irradiance"]


@pytest.mark.parametrize("name", G.GOLDEN_SCENES)
def test_oracle_matches_golden(name):
    want, last = load(name)
    got, got_last = G.oracle_run(name)
    assert got == want
    assert np.array_equal(got_last, last)


def test_half_rne_fixture_matches_reference_half_hpp_live():
    """When the reference tree is present (build container), re-run half.hpp."""
    exe = os.path.join(G.ROOT, "oracle", "_ref", "half_kat")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/half_kat not built (needs /root/reference)")
    import subprocess

    f = np.load(os.path.join(GOLDEN, "half_rne.npz"))
    r = subprocess.run([exe], input=f["inputs"].tobytes(), capture_output=True, check=True)
    assert np.array_equal(np.frombuffer(r.stdout, np.uint16), f["half_bits"])
