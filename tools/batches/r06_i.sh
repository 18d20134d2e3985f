# background rebuilds take turns (one scheduler for world and sun): rebuild progress at fast and slow frame rates, scene-update parity, continuous motion at C4 / C3
set -o pipefail
OUT=gpurun_out/r06_i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 python -u tools/motion_diag.py --seconds 20 --every 100 > $OUT/motion_fast.log 2>&1 || { echo "diag failed rc=$?"; tail -20 $OUT/motion_fast.log; exit 1; }
tail -2 $OUT/motion_fast.log
timeout -k 10 60 python -u tools/motion_diag.py --seconds 20 --every 20 --sleep 0.03 > $OUT/motion_slow.log 2>&1 || { echo "diag failed rc=$?"; tail -20 $OUT/motion_slow.log; exit 1; }
tail -2 $OUT/motion_slow.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_scene_update.py tests/test_gpu_cpp_node.py -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "PASS|FAIL|Error|error" $OUT/pytest.log | tail -30; exit 1; }
tail -1 $OUT/pytest.log
grep "continuous motion:" $OUT/pytest.log
timeout -k 10 400 python -u tools/refit_cost.py --continuous --frames 300 --config c4 c3 > $OUT/refit_bg.log 2>&1 || { echo "refit failed"; tail -20 $OUT/refit_bg.log; exit 1; }
grep config $OUT/refit_bg.log | cut -c1-1500
echo done
