# EXPERIMENT lighting compose latency: gather batch (cg2/cg4/cg8: sampleDDGI<GB>) and occupancy (cw6/cw8: waves_per_eu 6/8; cw8g2 both), interleaved twice, 200 launches each
set -o pipefail
OUT=gpurun_out/r06_l
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for v in shipped cg2 cg4 cg8 cw6 cw8 cw8g2; do
  if [[ $v == shipped ]]; then L=""; else L="ARK_DDGI_LIB=arkoserenderer_amd/lib_$v/libark_ddgi.so"; fi
  env TMPDIR=/tmp $L timeout -k 10 120 python3 tools/compose_bench.py --reps 200 > $OUT/compose_${v}_$rep.log 2>&1 || { echo "compose $v failed"; tail -5 $OUT/compose_${v}_$rep.log; exit 1; }
  echo "$rep $v $(tail -1 $OUT/compose_${v}_$rep.log)"
done
done
echo done
