"""The closed-form slot table and traversal order of k_probe_slots (ddgi_kernels.h:
slabRankOf, slotQueuePos), checked on the CPU against the plain construction (window
order, Z-slab compaction, stable bucket sort by x-z block) for every window of small
grids. Built with hipcc as host code (the header is shared with the kernels)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "arkoserenderer_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
def test_slot_table_and_order_closed_form(tmp_path):
    exe = str(tmp_path / "slot_order_check")
    src = os.path.join(ROOT, "tests", "cpp", "slot_order_check.cpp")
    r = subprocess.run([HIPCC, "-O1", "-std=c++17", "-I", CSRC, src, "-o", exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
