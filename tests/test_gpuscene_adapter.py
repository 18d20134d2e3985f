"""The C++ GpuScene -> ArkDdgiScene adapter (host/rendering/GpuScene.cpp), built with
g++ and run on the CPU: RT meshes and TLAS instances per LOD segment with hit masks by
blend mode (GpuScene.cpp:872-929), light data (GpuScene.cpp:790-858)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "arkoserenderer_amd", "host")


def test_gpuscene_adapter(tmp_path):
    exe = str(tmp_path / "adapter_test")
    src = os.path.join(ROOT, "tests", "cpp", "gpuscene_adapter_test.cpp")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", HOST, src, os.path.join(HOST, "rendering", "GpuScene.cpp"), "-o", exe],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
