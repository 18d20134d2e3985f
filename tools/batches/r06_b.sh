set -o pipefail
mkdir -p gpurun_out/r06_b
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_window_exchange.py tests/test_gpu_cpp_node.py tests/test_gpu_scene_update.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_b/pytest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 gpurun_out/r06_b/pytest.log; exit 1; }
tail -2 gpurun_out/r06_b/pytest.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_libm_parity.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r06_b/libm.log 2>&1 || { echo "libm tests failed rc=$?"; tail -40 gpurun_out/r06_b/libm.log; exit 1; }
tail -2 gpurun_out/r06_b/libm.log
timeout -k 10 500 python -u tools/shard_proxy.py --shards 1 8 --steps 30 --all-ranks --exchange --window 2048 > gpurun_out/r06_b/proxy_k2048.log 2>&1 || { echo proxy failed; tail -20 gpurun_out/r06_b/proxy_k2048.log; exit 1; }
tail -1 gpurun_out/r06_b/proxy_k2048.log
