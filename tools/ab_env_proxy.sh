#!/bin/bash
# GPU box: A/B over environment sets (each a space-separated list of VAR=value; "-" =
# none): the Z-slab shard proxy (slab 0 of 1/4/8, frames in flight) and the rolling
# windows (tools/window_proxy.py) per set. Stops at the first failure.
# Usage: tools/ab_env_proxy.sh <tag> <env set> <env set> ...
set -o pipefail
TAG=${1:-abe}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for setting in "$@"; do
  i=$((i+1))
  envs=""
  [[ "$setting" != "-" ]] && envs="$setting"
  env $envs timeout -k 10 200 python -u tools/shard_proxy.py --shards 1 4 8 --steps 100 > $OUT/proxy$i.log 2>&1 || { echo "proxy failed ($setting)"; tail -5 $OUT/proxy$i.log; exit 1; }
  env $envs timeout -k 10 200 python -u tools/window_proxy.py --repeats 2 > $OUT/win$i.log 2>&1 || { echo "window proxy failed ($setting)"; tail -5 $OUT/win$i.log; exit 1; }
  echo "$setting | $(tail -1 $OUT/proxy$i.log) | $(tail -1 $OUT/win$i.log)"
done
