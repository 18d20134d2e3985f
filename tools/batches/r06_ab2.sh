# EXPERIMENT refit ordering events, continuous motion C3 / C4 interleaved twice: new (events on the caller stream behind orderBegin), mark (own mark stream, ca49eaca), old (last operation's stream, d20676c4)
set -o pipefail
OUT=gpurun_out/r06_ab2
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
for v in new mark old; do
  if [[ $v == new ]]; then L=""; else L="ARK_DDGI_LIB=arkoserenderer_amd/lib_$v/libark_ddgi.so"; fi
  env TMPDIR=/tmp $L timeout -k 10 300 python3 -u tools/refit_cost.py --continuous --frames 300 --config c3 c4 --steps 20 > $OUT/refit_${v}_$rep.log 2>&1 || { echo "refit $v failed"; tail -5 $OUT/refit_${v}_$rep.log; exit 1; }
  echo "$rep $v $(grep -o '"config": "c[34]"\|"mrays_per_s_moving": [0-9.]*' $OUT/refit_${v}_$rep.log | tr '\n' ' ')"
done
done
echo done
