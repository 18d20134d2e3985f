# continuous-motion rebuild progress (diagnostic), refit cost under continuous motion at C4 / C3; counter passes of the sun's two structures
set -o pipefail
OUT=gpurun_out/r06_h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 90 python -u tools/motion_diag.py --seconds 40 > $OUT/motion_diag.log 2>&1 || { echo "diag failed rc=$?"; tail -20 $OUT/motion_diag.log; exit 1; }
tail -4 $OUT/motion_diag.log
timeout -k 10 400 python -u tools/refit_cost.py --continuous --frames 300 --config c4 c3 > $OUT/refit_bg.log 2>&1 || { echo "refit failed"; tail -20 $OUT/refit_bg.log; exit 1; }
grep config $OUT/refit_bg.log | cut -c1-1500
bash tools/prof_ab.sh r06_h_sunpmc --pmc "--sun-bvh world" "--sun-bvh light" || exit 1
echo done
