set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "city or real_ies" > gpurun_out/r01s3_pt2.log 2>&1; rc=$?; tail -3 gpurun_out/r01s3_pt2.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r01s3_pt2.log | head -20; exit 1; }
timeout -k 10 400 python -u tools/config_bench.py > gpurun_out/r01s3_configs.log 2>&1; tail -2 gpurun_out/r01s3_configs.log
