set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01s3_pt.log 2>&1 && tail -2 gpurun_out/r01s3_pt.log && \
bash tools/sweep_env.sh r01s3_ab4 "ARK_SHADOWS=split" "ARK_SHADOWS=pre" && \
timeout -k 10 300 python -u tools/shard_proxy.py --shards 8 > gpurun_out/r01s3_ab4/shard_pre.log 2>&1 && tail -n 1 gpurun_out/r01s3_ab4/shard_pre.log
