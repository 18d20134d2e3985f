# the eight-lane node refit: scene-update parity, continuous motion at C4 / C3; counter passes of the sun's two structures
set -o pipefail
OUT=gpurun_out/r06_g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scene_update.py tests/test_gpu_cpp_node.py -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "PASS|FAIL|Error|error" $OUT/pytest.log | tail -30; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python -u tools/refit_cost.py --continuous --frames 300 --config c4 c3 > $OUT/refit_bg.log 2>&1 || { echo "refit failed"; tail -20 $OUT/refit_bg.log; exit 1; }
grep config $OUT/refit_bg.log | cut -c1-1500
bash tools/prof_ab.sh r06_g_sunpmc --pmc "--sun-bvh world" "--sun-bvh light" || exit 1
echo done
