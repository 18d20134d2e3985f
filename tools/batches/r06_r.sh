# EXPERIMENT refit waves at s_setprio 3 (shipped) or not (lib_noprio), continuous motion at C4 / C3, interleaved twice
set -o pipefail
OUT=gpurun_out/r06_r
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for v in shipped noprio; do
  if [[ $v == shipped ]]; then L=""; else L="ARK_DDGI_LIB=arkoserenderer_amd/lib_$v/libark_ddgi.so"; fi
  env TMPDIR=/tmp $L timeout -k 10 400 python3 -u tools/refit_cost.py --continuous --frames 300 --config c4 c3 --steps 20 > $OUT/refit_${v}_$rep.log 2>&1 || { echo "refit $v failed"; tail -5 $OUT/refit_${v}_$rep.log; exit 1; }
  echo "$rep $v $(grep -o '"config": "c[34]"\|"mrays_per_s_moving": [0-9.]*' $OUT/refit_${v}_$rep.log | tr '\n' ' ')"
done
done
echo done
