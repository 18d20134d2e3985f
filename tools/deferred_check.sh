#!/bin/bash
# GPU box: deferred-update parity + bench A/B (serial vs deferred probe update).
set -o pipefail
OUT=gpurun_out/${1:-deferred}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 \
  || { echo "tests failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for d in 0 1 0 1; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-ao-bake --no-compose --deferred-update $d > $OUT/bench_$d.log 2>&1 \
    || { echo "bench failed rc=$?"; tail -20 $OUT/bench_$d.log; exit 1; }
  python -c "import json,sys; j=json.loads(open('$OUT/bench_$d.log').read().strip().splitlines()[-1]); print('deferred', $d, j['value'], j['ms_per_step'])"
done
