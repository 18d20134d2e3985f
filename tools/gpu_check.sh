#!/bin/bash
# One GPU-box pass: GPU parity suite, bench (N=1), rocprofv3 kernel stats + PMC passes.
# Every GPU step has its own time limit; the script stops at the first failure.
# Usage: tools/gpu_check.sh <tag> [--no-tests] [--no-prof]
set -o pipefail
TAG=${1:-check}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [[ " $* " != *" --no-tests "* ]]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
  tail -3 $OUT/pytest.log
fi
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
if [[ " $* " != *" --no-prof "* ]]; then
  bash tools/prof_run.sh $TAG/prof || exit 1
fi
echo "gpu_check done"
