set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01s3_pt.log 2>&1; rc=$?; tail -1 gpurun_out/r01s3_pt.log; [ $rc -eq 0 ] || { grep -E "assert|Error|FAILED" gpurun_out/r01s3_pt.log | head; exit 1; }
bash tools/sweep_env.sh r01s3_split "ARK_SHADE_SPLIT=0" "ARK_SHADE_SPLIT=1" "ARK_SHADE_SPLIT=0" "ARK_SHADE_SPLIT=1" && \
ARK_SHADE_SPLIT=0 timeout -k 10 300 python -u tools/shard_proxy.py --shards 8 > gpurun_out/r01s3_split/shard0.log 2>&1 && tail -n 1 gpurun_out/r01s3_split/shard0.log && \
timeout -k 10 300 python -u tools/shard_proxy.py --shards 8 > gpurun_out/r01s3_split/shard1.log 2>&1 && tail -n 1 gpurun_out/r01s3_split/shard1.log
