"""Prints the headline fields of bench.py JSON lines (last JSON line of each log).

    python tools/bench_line.py gpurun_out/<tag>/step*.log
"""
import json
import sys

for p in sys.argv[1:]:
    lines = [l for l in open(p).read().splitlines() if l.startswith("{")]
    if not lines:
        print(p, "no JSON line")
        continue
    j = json.loads(lines[-1])
    w = {k: (v["mrays_per_s"], v["ms_per_frame"]) for k, v in j.get("reference_windows", {}).items()}
    print(p, j["value"], j["ms_per_step"], j.get("kernels_ms"), w)
