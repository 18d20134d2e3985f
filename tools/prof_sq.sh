#!/bin/bash
# SQ / TCC counter passes (each its own run, --pmc only with --kernel-trace-free defaults).
set -o pipefail
TAG=${1:-sq}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs $*"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $OUT/sq1 -o run --output-format csv -- python3 $BENCH > $OUT/sq1.log 2>&1 || { echo "sq1 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD -d $OUT/sq2 -o run --output-format csv -- python3 $BENCH > $OUT/sq2.log 2>&1 || { echo "sq2 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE -d $OUT/tcc -o run --output-format csv -- python3 $BENCH > $OUT/tcc.log 2>&1 || { echo "tcc failed"; exit 1; }
echo "sq done"
