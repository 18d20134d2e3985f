set -o pipefail
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ao-bake > gpurun_out/r01s3_bench_compose.log 2>&1 && tail -1 gpurun_out/r01s3_bench_compose.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["lighting_compose"])'
