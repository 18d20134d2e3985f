#!/bin/bash
# GPU box: bench A/B over environment settings (one bench run per argument, each a
# space-separated list of VAR=value; "-" = no extra env). Short runs: no CPU baseline,
# no consumer lines.
# Usage: tools/ab_bench.sh <tag> [bench args --] <env set> <env set> ...
set -o pipefail
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
BARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-ao-bake --no-compose --no-windows"
if [[ " $* " == *" -- "* ]]; then
  while [[ "$1" != "--" ]]; do BARGS="$BARGS $1"; shift; done
  shift
fi
i=0
for setting in "$@"; do
  i=$((i+1))
  envs=""
  [[ "$setting" != "-" ]] && envs="$setting"
  env $envs timeout -k 10 240 python -u bench.py $BARGS > $OUT/run$i.log 2>&1 || { echo "bench failed ($setting) rc=$?"; tail -20 $OUT/run$i.log; exit 1; }
  python - "$OUT/run$i.log" "$setting" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps({"env": sys.argv[2], "value": j["value"], "ms_per_step": j["ms_per_step"], "kernels_ms": j["kernels_ms"], "per_ray": j.get("per_ray")}))
PY
done
