#!/bin/bash
# Runs on the GPU box: rocprofv3 kernel-trace stats, then PMC passes, each its own run
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; SQ and TCC counters in
# passes within the per-block limits), over a short C4 bench (no side lines).
# Usage: tools/prof_run.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-prof}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-windows --no-ao-bake --no-compose --no-configs $*"
# the byte passes also run the consumer lines (lighting compose, RT reflections)
BENCH_ALL="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-windows --no-ao-bake --no-configs $*"
run() { # name, then rocprofv3 options
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- python3 $BENCH > $OUT/$name.log 2>&1 || { echo "$name pass failed rc=$?"; tail -5 $OUT/$name.log; exit 1; }
}
run_all() { # name, then rocprofv3 options
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- python3 $BENCH_ALL > $OUT/$name.log 2>&1 || { echo "$name pass failed rc=$?"; tail -5 $OUT/$name.log; exit 1; }
}
run trace --kernel-trace --stats
run_all fetch --pmc FETCH_SIZE
run_all write --pmc WRITE_SIZE
run sq1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
run sq2 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD
run tcc --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE
echo "prof done"
