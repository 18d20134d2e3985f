#!/bin/bash
# Runs on the GPU box: rocprofv3 kernel-trace stats + two separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950) over a short bench.
# Usage: tools/prof_run.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-prof}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $BENCH > $OUT/trace.log 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $BENCH > $OUT/fetch.log 2>&1 || { echo "fetch pass failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $BENCH > $OUT/write.log 2>&1 || { echo "write pass failed rc=$?"; exit 1; }
echo "prof done"
