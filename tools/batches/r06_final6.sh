# the shipped library (ca49eaca): continuous motion at C4 / C3 against the static rate and a fresh build
set -o pipefail
OUT=gpurun_out/r06_final6
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/refit_cost.py --continuous --frames 300 --config c4 c3 --steps 20 > $OUT/refit_bg.log 2>&1 || { echo "refit failed"; tail -20 $OUT/refit_bg.log; exit 1; }
grep config $OUT/refit_bg.log | cut -c1-1800
echo done
