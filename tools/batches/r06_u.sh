# C4 and the C3 substitute at full size, every probe, two frames, against the oracle
set -o pipefail
OUT=gpurun_out/r06_u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -k every_probe -x -v -s --timeout 500 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "test failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
echo done
