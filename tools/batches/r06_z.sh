# one-off: the C5 substitute at full size, every probe, two frames, against the oracle (ARK_SLOW_TESTS=1)
set -o pipefail
OUT=gpurun_out/r06_z
mkdir -p $OUT
export TMPDIR=/tmp
export ARK_SLOW_TESTS=1
timeout -k 10 1100 python -u -m pytest tests/test_gpu_fullsize.py -k "every_probe and c5" -x -v -s --timeout 1050 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "test failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
echo done
