# moving instances at C4 / C3: device refit time, with and without background rebuilds; the sun A/B
set -o pipefail
OUT=gpurun_out/r06_f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/refit_cost.py --continuous --frames 300 --config c4 c3 > $OUT/refit_bg.log 2>&1 || { echo "refit failed"; tail -20 $OUT/refit_bg.log; exit 1; }
grep config $OUT/refit_bg.log | cut -c1-1500
timeout -k 10 300 python -u tools/refit_cost.py --continuous --frames 300 --config c4 --no-background > $OUT/refit_nobg.log 2>&1 || { echo "refit nobg failed"; tail -20 $OUT/refit_nobg.log; exit 1; }
grep config $OUT/refit_nobg.log | cut -c1-1500
timeout -k 10 400 python -u tools/sun_ab.py --reps 5 > $OUT/sun_ab.log 2>&1 || { echo "sun_ab failed"; tail -20 $OUT/sun_ab.log; exit 1; }
tail -1 $OUT/sun_ab.log | cut -c1-2000
