# one-off: C5 substitute every probe against the witness oracles (libm, no contraction, both), ARK_SLOW_TESTS=1
set -o pipefail
OUT=gpurun_out/r06_zb
mkdir -p $OUT
export TMPDIR=/tmp
export ARK_SLOW_TESTS=1
timeout -k 10 1100 python -u -m pytest tests/test_gpu_libm_parity.py -k "whole_grid and c5" -x -v -s --timeout 1050 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "test failed rc=$?"; grep -E "LIBM-SUMMARY|FAIL|Error" $OUT/pytest.log | tail -20; exit 1; }
grep "LIBM-SUMMARY" $OUT/pytest.log | cut -c1-400
tail -1 $OUT/pytest.log
echo done
