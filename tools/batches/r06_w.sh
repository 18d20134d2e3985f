# K = 2,048 frames in flight: window proxy rate and a kernel trace of 60 frames (where a 0.33-ms frame goes)
set -o pipefail
OUT=gpurun_out/r06_w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/window_proxy.py --frames 300 --repeats 3 --windows 2048 > $OUT/proxy.log 2>&1 || { echo proxy failed; tail -20 $OUT/proxy.log; exit 1; }
tail -2 $OUT/proxy.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python3 tools/window_proxy.py --frames 60 --repeats 1 --windows 2048 > $OUT/trace.log 2>&1 || { echo trace failed; tail -20 $OUT/trace.log; exit 1; }
echo done
