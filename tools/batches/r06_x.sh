# three frame sets, the slot table of a half-grid-or-smaller window on its own stream: GPU suite, window proxy K = 2,048 / 4,096, bench
set -o pipefail
OUT=gpurun_out/r06_x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "FAIL|Error" $OUT/pytest.log | tail -20; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u tools/window_proxy.py --frames 300 --repeats 3 > $OUT/proxy.log 2>&1 || { echo proxy failed; tail -20 $OUT/proxy.log; exit 1; }
tail -1 $OUT/proxy.log | cut -c1-400
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo bench failed; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['reference_windows']['K4096']['mrays_per_s'], d['reference_windows']['K2048']['mrays_per_s'], d['c5']['mrays_per_s'], d['c3']['mrays_per_s'])"
echo done
