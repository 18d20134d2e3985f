#!/bin/bash
# Runs bench.py once per environment setting string (tuning sweeps).
# Usage: tools/sweep_env.sh <tag> "A=1 B=2" "A=3" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-ao-bake > $OUT/bench_$i.log 2>&1 || { echo "bench [$cfg] failed rc=$?"; tail -5 $OUT/bench_$i.log; exit 1; }
  echo "[$cfg] $(tail -1 $OUT/bench_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernels_ms"], d["per_ray"].get("primary_lane_util"))')"
done
