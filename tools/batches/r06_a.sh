set -o pipefail
mkdir -p gpurun_out/r06_a
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06_a/pytest.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -40 gpurun_out/r06_a/pytest.log; exit 1; }
tail -3 gpurun_out/r06_a/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_a/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/r06_a/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-ao-bake > gpurun_out/r06_a/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/r06_a/bench.log; exit 1; }
tail -1 gpurun_out/r06_a/bench.log | cut -c1-600
