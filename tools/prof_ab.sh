#!/bin/bash
# GPU box: rocprofv3 kernel-trace stats and (optionally) FETCH_SIZE / WRITE_SIZE passes of
# a short serial C4 bench (--serial-frames: kernels do not overlap, so each kernel's
# duration is its own) per setting: "VAR=value ..." environment words (e.g.
# ARK_DDGI_LIB=<variant library>) and/or bench.py arguments ("-" = none).
# Usage: tools/prof_ab.sh <tag> [--pmc] <setting> <setting> ...
set -o pipefail
TAG=${1:-pab}; shift
PMC=0
if [[ "$1" == "--pmc" ]]; then PMC=1; shift; fi
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-windows --no-ao-bake --no-compose --no-configs --serial-frames"
i=0
for setting in "$@"; do
  i=$((i+1))
  envs="TMPDIR=/tmp"; bargs=""
  if [[ "$setting" != "-" ]]; then
    for w in $setting; do if [[ "$w" == *=* && "$w" != --* ]]; then envs="$envs $w"; else bargs="$bargs $w"; fi; done
  fi
  echo "$i: $setting" >> $OUT/sets.txt
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t$i -o run --output-format csv -- python3 $BENCH $bargs > $OUT/t$i.log 2>&1 || { echo "trace $i failed"; tail -5 $OUT/t$i.log; exit 1; }
  if [[ $PMC == 1 ]]; then
    env $envs timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/f$i -o run --output-format csv -- python3 $BENCH $bargs > $OUT/f$i.log 2>&1 || { echo "fetch $i failed"; tail -5 $OUT/f$i.log; exit 1; }
    env $envs timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/w$i -o run --output-format csv -- python3 $BENCH $bargs > $OUT/w$i.log 2>&1 || { echo "write $i failed"; tail -5 $OUT/w$i.log; exit 1; }
  fi
  echo "done $i: $setting"
done
