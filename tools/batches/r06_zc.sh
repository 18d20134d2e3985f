# one-off: the C5 whole grid's witness flips classified (geometric vs radiance only), frame 0, libm and no-contraction witnesses
set -o pipefail
OUT=gpurun_out/r06_zc
mkdir -p $OUT
export TMPDIR=/tmp
for v in libm nocontract; do
  timeout -k 10 400 python -u tools/flip_breakdown.py --config c5 --variant $v > $OUT/flips_$v.log 2>&1 || { echo "breakdown $v failed"; tail -20 $OUT/flips_$v.log; exit 1; }
  tail -1 $OUT/flips_$v.log
done
echo done
