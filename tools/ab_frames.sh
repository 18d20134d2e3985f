#!/bin/bash
# GPU box: A/B of frame-pipelining settings over environment sets (each a space-separated
# list of VAR=value; "-" = none): per set, the Z-slab shard proxy (slab 0 of 1/4/8) and a
# short bench with the reference windows (K = 4096 / 2048). Stops at the first failure.
# Usage: tools/ab_frames.sh <tag> <env set> <env set> ...
set -o pipefail
TAG=${1:-abf}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for setting in "$@"; do
  i=$((i+1))
  envs=""
  [[ "$setting" != "-" ]] && envs="$setting"
  env $envs timeout -k 10 240 python -u tools/shard_proxy.py --shards 1 4 8 --steps 60 > $OUT/proxy$i.log 2>&1 || { echo "proxy failed ($setting) rc=$?"; tail -20 $OUT/proxy$i.log; exit 1; }
  env $envs timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ao-bake --no-compose > $OUT/bench$i.log 2>&1 || { echo "bench failed ($setting) rc=$?"; tail -20 $OUT/bench$i.log; exit 1; }
  python - "$OUT/proxy$i.log" "$OUT/bench$i.log" "$setting" <<'PY'
import json, sys
p = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
b = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
w = b.get("reference_windows", {})
print(json.dumps({"env": sys.argv[3], "proxy_ms": {str(r["shards"]): r["ms_per_step"] for r in p if "shards" in r},
                  "c4": b["value"], "k4096_ms": w.get("K4096", {}).get("ms_per_frame"), "k2048_ms": w.get("K2048", {}).get("ms_per_frame")}))
PY
done
