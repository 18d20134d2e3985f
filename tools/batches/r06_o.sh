# refits reach only the moved instances' nodes (node masks, records transformed in the leaf pass): scene-update parity + partial-vs-full digests, C++ node, shared scenes; continuous motion at C4 / C3; trace
set -o pipefail
OUT=gpurun_out/r06_o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_scene_update.py tests/test_gpu_cpp_node.py tests/test_gpu_sharded.py -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "PASS|FAIL|Error|error" $OUT/pytest.log | tail -30; exit 1; }
tail -1 $OUT/pytest.log
grep "frames in flight:" $OUT/pytest.log
timeout -k 10 500 python -u tools/refit_cost.py --continuous --frames 300 --config c4 c3 --steps 20 > $OUT/refit_bg.log 2>&1 || { echo "refit failed"; tail -20 $OUT/refit_bg.log; exit 1; }
grep config $OUT/refit_bg.log | cut -c1-1800
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/refit_cost.py --continuous --frames 60 --config c4 --steps 10 > $OUT/trace.log 2>&1 || { echo "trace failed rc=$?"; tail -20 $OUT/trace.log; exit 1; }
echo done
