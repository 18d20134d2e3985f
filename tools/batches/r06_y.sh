# EXPERIMENT A/B on one box: early slot tables on three frame sets (shipped tree) against two sets (lib_prev = HEAD before), window proxy K = 4,096 / 2,048, interleaved three times
set -o pipefail
OUT=gpurun_out/r06_y
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
for v in new prev; do
  if [[ $v == new ]]; then L=""; else L="ARK_DDGI_LIB=arkoserenderer_amd/lib_prev/libark_ddgi.so"; fi
  env TMPDIR=/tmp $L timeout -k 10 200 python3 -u tools/window_proxy.py --frames 300 --repeats 3 > $OUT/proxy_${v}_$rep.log 2>&1 || { echo "proxy $v failed"; tail -5 $OUT/proxy_${v}_$rep.log; exit 1; }
  echo "$rep $v $(tail -1 $OUT/proxy_${v}_$rep.log)"
done
done
echo done
