# end of round 6, the shipped library (ca49eaca): rocprofv3 kernel stats + PMC + SQ passes (summaries of this build into profiles/), the driver's bench command reading them, kernel-trace stats of that command
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_check.sh r06_final5 --no-tests || exit 1
OUT=gpurun_out/r06_final5
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/bench_trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || { echo "bench trace failed"; tail -5 $OUT/bench_trace.log; exit 1; }
echo done
