set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01s3_pt.log 2>&1; rc=$?; tail -1 gpurun_out/r01s3_pt.log; [ $rc -eq 0 ] || { grep -E "assert|Error|FAILED" gpurun_out/r01s3_pt.log | head; exit 1; }
