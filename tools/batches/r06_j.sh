# continuous motion at C4: kernel + HIP runtime trace of 60 moving frames (where the 4.6 ms per frame go); continuous runs at C4 / C3 against a fresh build of the final transforms
set -o pipefail
OUT=gpurun_out/r06_j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/refit_cost.py --continuous --frames 60 --config c4 --steps 10 > $OUT/trace.log 2>&1 || { echo "trace failed rc=$?"; tail -20 $OUT/trace.log; exit 1; }
grep config $OUT/trace.log | cut -c1-1200
timeout -k 10 500 python -u tools/refit_cost.py --continuous --frames 300 --config c4 c3 --steps 20 > $OUT/refit_bg.log 2>&1 || { echo "refit failed"; tail -20 $OUT/refit_bg.log; exit 1; }
grep config $OUT/refit_bg.log | cut -c1-1800
echo done
