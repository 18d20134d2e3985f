#!/bin/bash
# Runs bench.py once per value of an environment variable (tuning sweeps).
# Usage: tools/sweep.sh <tag> <VAR> <v1> [v2 ...]
set -o pipefail
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in "$@"; do
  env $VAR=$v timeout -k 10 240 python -u bench.py --no-cpu-baseline > $OUT/bench_$v.log 2>&1 || { echo "bench $VAR=$v failed rc=$?"; tail -5 $OUT/bench_$v.log; exit 1; }
  echo "$VAR=$v $(tail -1 $OUT/bench_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["kernels_ms"], d["per_ray"], d["config"]["bvh_nodes"])')"
done
