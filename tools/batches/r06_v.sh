# windowed Z-slab exchange proxy at the reference's node cap K = 4,096, P = 8 (K = 2,048 in r06_b)
set -o pipefail
OUT=gpurun_out/r06_v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/shard_proxy.py --shards 1 8 --steps 30 --all-ranks --exchange --window 4096 > $OUT/proxy_k4096.log 2>&1 || { echo proxy failed; tail -20 $OUT/proxy_k4096.log; exit 1; }
tail -1 $OUT/proxy_k4096.log
echo done
