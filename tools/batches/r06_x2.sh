# K = 2,048 with early slot tables: proxy rate and kernel trace
set -o pipefail
OUT=gpurun_out/r06_x2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/window_proxy.py --frames 300 --repeats 3 --windows 2048 > $OUT/proxy.log 2>&1 || { echo proxy failed; tail -20 $OUT/proxy.log; exit 1; }
tail -2 $OUT/proxy.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python3 tools/window_proxy.py --frames 60 --repeats 1 --windows 2048 > $OUT/trace.log 2>&1 || { echo trace failed; tail -20 $OUT/trace.log; exit 1; }
echo done
