#!/bin/bash
# GPU box: runs a list of experiment steps (one shell command per line of a steps
# file), each under its own time limit, logging to gpurun_out/<tag>/step<N>.log.
# A step that fails with an ordinary error is recorded and the batch goes on; a
# time limit (124/137), an abort (134) or a segfault (139) ends the batch (nothing
# more runs on the GPU after a fault or a hang).
# Usage: tools/batch.sh <tag> <steps file> [seconds per step]
TAG=$1; STEPS=$2; LIMIT=${3:-400}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
while IFS= read -r cmd; do
  [[ -z "$cmd" || "$cmd" == \#* ]] && continue
  i=$((i+1))
  echo "[$i] $cmd" >> $OUT/steps.txt
  timeout -k 10 $LIMIT bash -c "$cmd" > $OUT/step$i.log 2>&1
  rc=$?
  echo "[$i] rc=$rc" >> $OUT/steps.txt
  echo "step $i rc=$rc: $cmd"
  if [[ $rc == 124 || $rc == 137 || $rc == 134 || $rc == 139 ]]; then echo "stopping after rc $rc"; exit $rc; fi
done < $STEPS
