# EXPERIMENTS (1) triangle records padded 48 -> 64 B (lib_t64): the traversal's sensitivity to triangle bytes, beside round 5's 80 -> 128-B nodes (+15 %): interleaved C4 A/B and FETCH/WRITE counter passes (serial frames); (2) lighting compose tile shapes 16x16 (shipped) / 32x8 (lib_c32) / 64x4 (lib_c64): time and counter traffic of tools/compose_bench.py
set -o pipefail
OUT=gpurun_out/r06_c
mkdir -p $OUT
export TMPDIR=/tmp
T64=ARK_DDGI_LIB=arkoserenderer_amd/lib_t64/libark_ddgi.so
bash tools/ab_bench.sh r06_c_ab $T64 - $T64 - $T64 - || exit 1
bash tools/prof_ab.sh r06_c_pmc --pmc - $T64 || exit 1
for v in shipped c32 c64; do
  if [[ $v == shipped ]]; then L=""; else L="ARK_DDGI_LIB=arkoserenderer_amd/lib_$v/libark_ddgi.so"; fi
  env TMPDIR=/tmp $L timeout -k 10 120 python3 tools/compose_bench.py > $OUT/compose_$v.log 2>&1 || { echo "compose $v failed"; tail -5 $OUT/compose_$v.log; exit 1; }
  tail -1 $OUT/compose_$v.log
  env TMPDIR=/tmp $L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/ct_$v -o run --output-format csv -- python3 tools/compose_bench.py > $OUT/ct_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  env TMPDIR=/tmp $L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/cf_$v -o run --output-format csv -- python3 tools/compose_bench.py > $OUT/cf_$v.log 2>&1 || { echo "fetch $v failed"; exit 1; }
  env TMPDIR=/tmp $L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/cw_$v -o run --output-format csv -- python3 tools/compose_bench.py > $OUT/cw_$v.log 2>&1 || { echo "write $v failed"; exit 1; }
done
echo done1
