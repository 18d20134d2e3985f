#!/bin/bash
# One GPU-box pass: GPU parity suite, rocprofv3 kernel stats + PMC + SQ passes of this
# build (summarised into profiles/ on the box, so the bench below reads the traffic
# of its own build; copies land in gpurun_out/<tag>/profiles), then bench.py (N=1).
# Every GPU step has its own time limit; the script stops at the first failure.
# Usage: tools/gpu_check.sh <tag> [--no-tests] [--no-prof]
set -o pipefail
TAG=${1:-check}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT/profiles
export TMPDIR=/tmp
if [[ " $* " != *" --no-tests "* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
    || { echo "gpu tests failed rc=$?"; tail -30 $OUT/pytest.log; exit 1; }
  tail -3 $OUT/pytest.log
fi
if [[ " $* " != *" --no-prof "* ]]; then
  bash tools/prof_run.sh $TAG/prof || exit 1
  python3 tools/pmc_summary.py $OUT/prof $TAG --latest > $OUT/pmc_summary.log 2>&1 || { echo "pmc summary failed"; exit 1; }
  python3 tools/sq_summary.py $OUT/prof $TAG --json --latest > profiles/${TAG}_sq.txt 2>&1 || { echo "sq summary failed"; exit 1; }
  cp profiles/${TAG}_* profiles/latest_pmc.json profiles/latest_sq.json $OUT/profiles/
fi
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
echo "gpu_check done"
