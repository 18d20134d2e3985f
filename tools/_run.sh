set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01s3_pt.log 2>&1 && tail -2 gpurun_out/r01s3_pt.log && \
bash tools/sweep_env.sh r01s3_ab5 "ARK_SUBWINDOWS=1" "ARK_SUBWINDOWS=2" "ARK_SUBWINDOWS=3" "ARK_SUBWINDOWS=4" && \
timeout -k 10 300 python -u tools/shard_proxy.py --shards 8 > gpurun_out/r01s3_ab5/shard_s2.log 2>&1 && tail -n 1 gpurun_out/r01s3_ab5/shard_s2.log && \
ARK_SUBWINDOWS=4 timeout -k 10 300 python -u tools/shard_proxy.py --shards 8 > gpurun_out/r01s3_ab5/shard_s4.log 2>&1 && tail -n 1 gpurun_out/r01s3_ab5/shard_s4.log
