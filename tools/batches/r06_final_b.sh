# end of round 6, frozen library: rocprofv3 kernel stats + PMC + SQ passes (summaries of this build into profiles/), the driver's bench command reading them, kernel-trace stats of that command, the sun-turn rates at 20 steps
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_check.sh r06_final2 --no-tests || exit 1
OUT=gpurun_out/r06_final2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/bench_trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || { echo "bench trace failed"; tail -5 $OUT/bench_trace.log; exit 1; }
tail -1 $OUT/bench_trace.log | cut -c1-300
timeout -k 10 300 python3 -u tools/refit_cost.py --sun-turn --config c4 --steps 20 > $OUT/sun_turn.log 2>&1 || { echo "sun turn failed"; tail -5 $OUT/sun_turn.log; exit 1; }
tail -1 $OUT/sun_turn.log
echo done
