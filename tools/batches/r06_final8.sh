# end of round 6, the shipped library (5ebc5676): rocprofv3 kernel stats + PMC + SQ passes (summaries of this build into profiles/), the driver's bench command reading them, kernel-trace stats of that command
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_check.sh r06_final8 --no-tests || exit 1
OUT=gpurun_out/r06_final8
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/bench_trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || { echo "bench trace failed"; tail -5 $OUT/bench_trace.log; exit 1; }

timeout -k 10 500 python -u tools/refit_cost.py --continuous --frames 300 --config c4 c3 --steps 20 > $OUT/refit_bg.log 2>&1 || { echo "refit failed"; tail -20 $OUT/refit_bg.log; exit 1; }
grep config $OUT/refit_bg.log | cut -c1-600
echo done
