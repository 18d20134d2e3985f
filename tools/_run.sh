set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r01s3_sortprof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ao-bake --no-compose > gpurun_out/r01s3_sortprof.log 2>&1 && cut -d, -f1-4 gpurun_out/r01s3_sortprof/run_kernel_stats.csv | head -12
