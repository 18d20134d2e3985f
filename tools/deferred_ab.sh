#!/bin/bash
# GPU box: bench A/B of the deferred probe update (env settings per run as arguments).
set -o pipefail
OUT=gpurun_out/${1:-deferred_ab}; shift
mkdir -p $OUT
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ao-bake --no-compose > $OUT/bench_$i.log 2>&1 \
    || { echo "bench failed rc=$?"; tail -20 $OUT/bench_$i.log; exit 1; }
  grep "ark_ddgi: stream" $OUT/bench_$i.log | head -1
  python -c "import json,sys; j=json.loads(open('$OUT/bench_$i.log').read().strip().splitlines()[-1]); print('$cfg', j['value'], j['ms_per_step'])"
done
