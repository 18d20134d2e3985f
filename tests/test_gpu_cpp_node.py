"""The C++ drop-in DDGINode (RenderPipelineNode + Registry on the HIP backend,
driven headless) produces exactly what the Python mirror of the reference's
execute lambda produces — including a pipeline rebuild that must carry the DDGI
history through the Registry (Registry.cpp:120-150)."""
import os
import subprocess

import numpy as np
import pytest

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
from arkoserenderer_amd import scene as S
import scenes

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "arkoserenderer_amd", "bin", "ddgi_headless")


def _python_run(sc, grid, cfg, frames, zfar, exposure, rebuild=-1):
    node = D.DDGINode(cfg)
    assert node.construct(sc, grid, zfar, **exposure)
    for f in range(frames):
        if f == rebuild:  # reconstruct: atlases and the window index persist, offsets restart at 0
            node.ctx.synchronize()
            node.ctx.write(abi.ARK_DDGI_PROBE_OFFSETS, np.zeros(node.ctx.size(abi.ARK_DDGI_PROBE_OFFSETS) // 4, np.float32))
        node.execute(D.AppState(f))
    node.ctx.synchronize()
    return {k: node.ctx.read(w) for k, w in (("irr", abi.ARK_DDGI_ATLAS_IRRADIANCE), ("vis", abi.ARK_DDGI_ATLAS_VISIBILITY),
                                              ("off", abi.ARK_DDGI_PROBE_OFFSETS), ("surf", abi.ARK_DDGI_SURFELS))}


@pytest.mark.parametrize("rebuild", [-1, 2])
def test_cpp_node_matches_python_host(tmp_path, rebuild):
    sc = scenes.features_scene()
    grid = D.ProbeGrid((6, 4, 6), (0.7, 0.7, 0.7), (-1.75, 0.25, -1.75))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=100, max_rays_per_probe=512, max_probe_updates=100)
    exposure = dict(light_pre_exposure=0.5, ambient_illuminance=0.1, environment_brightness=0.8)
    path = str(tmp_path / "features.arkscn")
    sc.save_binary(path)
    out = str(tmp_path / "cpp")
    cmd = [EXE, "--scene", path, "--grid", "6", "4", "6", "--spacing", "0.7", "0.7", "0.7", "--origin", "-1.75", "0.25", "-1.75",
           "--rays", "64", "--updates", "100", "--frames", "5", "--zfar", "100", "--exposure", "0.5", "--env", "0.8",
           "--ambient", "0.1", "--offsets", "1", "--rebuild-at", str(rebuild), "--out", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    py = _python_run(sc, grid, cfg, 5, 100.0, exposure, rebuild)
    for k, dt in (("irr", np.uint16), ("vis", np.uint16), ("off", np.float32)):
        got = np.fromfile(out + "." + k, dtype=dt)
        assert np.array_equal(got, py[k]), k


def _headless(tmp_path, tag, extra):
    sc = scenes.features_scene()
    path = str(tmp_path / "features.arkscn")
    if not os.path.exists(path):
        sc.save_binary(path)
    out = str(tmp_path / tag)
    cmd = [EXE, "--scene", path, "--grid", "6", "4", "6", "--spacing", "0.7", "0.7", "0.7", "--origin", "-1.75", "0.25", "-1.75",
           "--rays", "64", "--updates", "100", "--frames", "4", "--zfar", "100", "--exposure", "0.5", "--env", "0.8",
           "--ambient", "0.1", "--offsets", "1", "--out", out] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return out, r.stdout


@pytest.mark.parametrize("updates", [100, 144])
@pytest.mark.parametrize("shards", [2, 3])
def test_cpp_zslab_device_copy_exchange_equals_unsharded(tmp_path, shards, updates):
    """C++ Z-slab ranks (DDGINode::setSlabExchange + ark_ddgi_update_overlapped):
    P contexts in one process, exchanging on a side stream: a rolling window of 100 of
    the 144 probes moves only the window's tiles (ark_ddgi_pack_window / _unpack_window),
    the whole grid (144) the row bands by device copies; every context ends with the
    unsharded atlases, bit for bit, and the owners' offsets merge to the unsharded
    offsets."""
    ref, _ = _headless(tmp_path, f"ref{updates}", ["--updates", str(updates)])
    got, log = _headless(tmp_path, f"s{shards}_{updates}", ["--shards", str(shards), "--updates", str(updates)])
    assert f"{shards} Z-slab ranks, device-copy exchange" in log
    for k, dt in (("irr", np.uint16), ("vis", np.uint16), ("off", np.float32)):
        assert np.array_equal(np.fromfile(got + "." + k, dtype=dt), np.fromfile(ref + "." + k, dtype=dt)), k


def test_cpp_rccl_exchange_one_rank(tmp_path):
    """The RCCL path of the C++ exchange (ncclCommInitRank from a shared unique id,
    in-place ncclAllGather of both bands in one group on a side stream) with a
    1-rank communicator: the run equals the unsharded one."""
    ref, _ = _headless(tmp_path, "ref", [])
    got, log = _headless(tmp_path, "rccl", ["--world", "1", "--rank", "0", "--nccl-id", str(tmp_path / "nccl.id")])
    assert "rccl exchange" in log
    for k, dt in (("irr", np.uint16), ("vis", np.uint16), ("off", np.float32)):
        assert np.array_equal(np.fromfile(got + "." + k, dtype=dt), np.fromfile(ref + "." + k, dtype=dt)), k


def test_cpp_rccl_exchange_watchdog_deadline(tmp_path):
    """Failure detection of the C++ exchange: a 1-rank communicator whose
    side stream is stalled for 1.5 s (a bounded kernel) under a 0.2 s deadline. Frame
    3's exchange waits for frame 0's all-gather, the watchdog polls the event and
    ncclCommGetAsyncError, fires at the deadline, and the default failure path aborts
    the communicator, logs an Error and ends the process with exit code 14 (the stall
    kernel is allowed to finish first, so nothing is left running on the GPU)."""
    sc = scenes.features_scene()
    path = str(tmp_path / "features.arkscn")
    sc.save_binary(path)
    cmd = [EXE, "--scene", path, "--grid", "6", "4", "6", "--spacing", "0.7", "0.7", "0.7", "--origin", "-1.75", "0.25", "-1.75",
           "--rays", "64", "--updates", "100", "--frames", "4", "--zfar", "100", "--out", str(tmp_path / "dl"),
           "--world", "1", "--rank", "0", "--nccl-id", str(tmp_path / "nccl.id"), "--exchange-deadline-test"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 14, (r.returncode, r.stdout, r.stderr)
    assert "watchdog fired: RcclSlabExchange frame n-3: not complete after" in r.stdout, r.stdout
    assert "[error] z-slab exchange failed, exiting" in r.stderr.lower(), r.stderr


def test_cpp_rccl_rendezvous_ignores_stale_id(tmp_path):
    """Rank 0 replaces an id file left by an earlier run: a stale file
    holding garbage sits at the path before the 1-rank run starts; the run must still
    initialise its communicator and equal the unsharded run."""
    ref, _ = _headless(tmp_path, "ref", [])
    stale = tmp_path / "nccl.id"
    stale.write_bytes(b"\xab" * 128)
    got, log = _headless(tmp_path, "rccl", ["--world", "1", "--rank", "0", "--nccl-id", str(stale), "--nccl-nonce", "run-2"])
    assert "rccl exchange" in log
    assert stale.read_bytes().endswith(b"run-2")
    for k, dt in (("irr", np.uint16), ("vis", np.uint16)):
        assert np.array_equal(np.fromfile(got + "." + k, dtype=dt), np.fromfile(ref + "." + k, dtype=dt)), k


def _frame_script(path, frames, instances):
    """ARKFRM1 (ddgi_headless --frame-script): per frame the exposure, the managed sun
    (colour, intensity, forward) and spots, and the instances' transforms when moved."""
    import struct

    with open(path, "wb") as fh:
        fh.write(b"ARKFRM1\0" + struct.pack("<II", len(frames), instances))
        for fr in frames:
            fh.write(struct.pack("<f", fr["exposure"]))
            sun = fr["sun"]
            fh.write(struct.pack("<i7f", 1 if sun else 0, *((sun["color"] + (sun["intensity"],) + sun["forward"]) if sun else (0.0,) * 7)))
            fh.write(struct.pack("<I", len(fr["spots"])))
            for sl in fr["spots"]:
                fh.write(struct.pack("<17fi", *sl["color"], sl["intensity"], *sl["forward"], *sl["right"], *sl["up"], *sl["position"],
                                     sl["cone"], sl["ies"]))
            M = fr.get("transforms")
            fh.write(struct.pack("<I", 0 if M is None else 1))
            if M is not None:
                fh.write(np.ascontiguousarray(M, np.float32).tobytes())


def _pre(c, intensity, pre):
    # GpuScene::updateLightData: colour * intensity * lightPreExposure, in fp32, left to right
    return tuple(float(np.float32(np.float32(x) * np.float32(intensity)) * np.float32(pre)) for x in c)


def test_cpp_node_per_frame_lights_and_instances(tmp_path):
    """the C++ DDGINode re-reads GpuScene's lights with the camera's
    current exposure every frame (GpuScene.cpp:792-858) and refits when an instance
    moved (:872-1009). Script: the exposure changes at frames 1 and 3, a spot moves at
    frame 2, the sun rotates at frame 3, the box instance moves at frames 2 and 4 (the
    mirrored box loses its mirroring at 4). The C++ run equals the Python mirror fed the
    same per-frame inputs (ark_ddgi_set_lights / _set_instances), bit for bit."""
    sc = scenes.features_scene()
    grid = D.ProbeGrid((6, 4, 6), (0.7, 0.7, 0.7), (-1.75, 0.25, -1.75))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=100, max_rays_per_probe=512, max_probe_updates=100)
    sun_c, sun_i = (1.0, 0.95, 0.85), 2.0
    d0 = tuple(float(x) for x in np.array([0.3, -1.0, -0.4]) / np.linalg.norm([0.3, -1.0, -0.4]))
    d1 = tuple(float(x) for x in np.array([-0.4, -0.9, 0.2]) / np.linalg.norm([-0.4, -0.9, 0.2]))
    spot_a = dict(color=(1.0, 0.8, 0.6), intensity=30.0, forward=(0.0, -1.0, 0.0), right=(1.0, 0.0, 0.0), up=(0.0, 0.0, 1.0),
                  position=(0.0, 2.9, 0.0), cone=1.6, ies=2)
    spot_b = dict(spot_a, forward=(0.6, -0.8, 0.0), right=(0.0, 0.0, 1.0), up=(0.8, 0.6, 0.0), position=(-1.8, 2.5, 0.2), intensity=12.0)
    spot_a2 = dict(spot_a, position=(0.5, 2.7, -0.6), forward=(0.28, -0.96, 0.0), right=(0.96, 0.28, 0.0))
    inst0 = sc.instances.copy()
    M0 = inst0["object_to_world"].reshape(-1, 3, 4).copy()

    def moved(step):
        M = M0.copy()
        M[3, :, 3] += np.float32(0.2 * step)
        if step >= 2:
            M[4, :, :3] = np.diag([1.0, 1.2, 1.0]).astype(np.float32)
        return M.reshape(-1, 12)

    frames = [
        dict(exposure=0.5, sun=dict(color=sun_c, intensity=sun_i, forward=d0), spots=[spot_a, spot_b]),
        dict(exposure=0.8, sun=dict(color=sun_c, intensity=sun_i, forward=d0), spots=[spot_a, spot_b]),
        dict(exposure=0.8, sun=dict(color=sun_c, intensity=sun_i, forward=d0), spots=[spot_a2, spot_b], transforms=moved(1)),
        dict(exposure=1.3, sun=dict(color=sun_c, intensity=sun_i, forward=d1), spots=[spot_a2, spot_b]),
        dict(exposure=1.3, sun=dict(color=sun_c, intensity=sun_i, forward=d1), spots=[spot_a2], transforms=moved(2)),
    ]
    scene_path, script = str(tmp_path / "features.arkscn"), str(tmp_path / "frames.arkfrm")
    sc.save_binary(scene_path)
    _frame_script(script, frames, len(inst0))
    out = str(tmp_path / "cpp")
    cmd = [EXE, "--scene", scene_path, "--grid", "6", "4", "6", "--spacing", "0.7", "0.7", "0.7", "--origin", "-1.75", "0.25", "-1.75",
           "--rays", "64", "--updates", "100", "--frames", str(len(frames)), "--zfar", "100", "--exposure", "0.5", "--env", "0.8",
           "--ambient", "0.1", "--offsets", "1", "--frame-script", script, "--out", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    # the Python mirror: the same node, the same per-frame inputs
    node = D.DDGINode(cfg)
    assert node.construct(sc, grid, 100.0, light_pre_exposure=0.5, ambient_illuminance=0.1, environment_brightness=0.8)
    for f, fr in enumerate(frames):
        pre = fr["exposure"]
        s = fr["sun"]
        sun = (_pre(s["color"], s["intensity"], pre), s["forward"])
        spots = [S.SpotLight(_pre(x["color"], x["intensity"], pre), x["forward"], x["right"], x["up"], x["position"],
                             float(np.float32(x["cone"]) / np.float32(2.0)), x["ies"]) for x in fr["spots"]]
        node.ctx.set_lights(sun, spots)
        if "transforms" in fr:
            inst = inst0.copy()
            inst["object_to_world"] = fr["transforms"]
            node.ctx.set_instances(inst)
        node.exposure.update(light_pre_exposure=pre)
        node.execute(D.AppState(f))
    node.ctx.synchronize()
    py = {k: node.ctx.read(w) for k, w in (("irr", abi.ARK_DDGI_ATLAS_IRRADIANCE), ("vis", abi.ARK_DDGI_ATLAS_VISIBILITY),
                                            ("off", abi.ARK_DDGI_PROBE_OFFSETS))}
    for k, dt in (("irr", np.uint16), ("vis", np.uint16), ("off", np.float32)):
        assert np.array_equal(np.fromfile(out + "." + k, dtype=dt), py[k]), k
