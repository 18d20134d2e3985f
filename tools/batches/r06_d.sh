# the moving-instances rework (stream-ordered refits, light-space refit, background rebuilds): the GPU suite, smoke, refit_cost --continuous at C3 and C4
set -o pipefail
mkdir -p gpurun_out/r06_d
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r06_d/pytest.log 2>&1 || { echo "gpu tests failed rc=$?"; grep -E "PASS|FAIL|Error|error" gpurun_out/r06_d/pytest.log | tail -30; exit 1; }
tail -2 gpurun_out/r06_d/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_d/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/r06_d/smoke.log; exit 1; }
timeout -k 10 600 python -u tools/refit_cost.py --continuous --frames 300 --config c3 c4 > gpurun_out/r06_d/refit_continuous.log 2>&1 || { echo refit failed; tail -20 gpurun_out/r06_d/refit_continuous.log; exit 1; }
grep config gpurun_out/r06_d/refit_continuous.log
