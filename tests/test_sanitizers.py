"""Sanitizer runs of the host code on the path (sanitizers / race
detection), CPU only: the oracle (three frames with probe offsets, the AO bake), the
soup generator and the BVH2 -> BVH8 builder with its structural check, built from
tests/cpp/sanitize_test.cpp with g++ under AddressSanitizer + UndefinedBehaviorSanitizer
(any report aborts) and, separately, ThreadSanitizer (the oracle's and the builder's
worker threads)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = [
    os.path.join(ROOT, "tests", "cpp", "sanitize_test.cpp"),
    os.path.join(ROOT, "oracle", "ddgi_oracle.cpp"),
    os.path.join(ROOT, "arkoserenderer_amd", "csrc", "bvh_builder.cpp"),
    os.path.join(ROOT, "arkoserenderer_amd", "csrc", "scene_gen.cpp"),
]


@pytest.mark.parametrize("flags", [["-fsanitize=address,undefined", "-fno-sanitize-recover=all"], ["-fsanitize=thread"]],
                         ids=["asan_ubsan", "tsan"])
def test_host_code_under_sanitizers(tmp_path, flags):
    exe = str(tmp_path / "sanitize_test")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", "-ffp-contract=off",
           "-I", os.path.join(ROOT, "arkoserenderer_amd", "csrc")] + flags + SOURCES + ["-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "OK" in r.stdout
    assert "ERROR: " not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr
