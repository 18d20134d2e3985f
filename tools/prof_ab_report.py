"""Table of tools/prof_ab.sh output: per environment set, the average duration of each
path kernel (serial run) and, with --pmc passes, its HBM bytes per launch
((2 FETCH_SIZE + WRITE_SIZE) KiB, MI355X_MICROARCH.md §HBM).

    python tools/prof_ab_report.py gpurun_out/<tag> [kernel ...]
"""
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main():
    d = sys.argv[1]
    want = sys.argv[2:] or ["k_trace", "k_shadow_gen", "k_shadow_bin_scan", "k_shadow_scatter", "k_trace_shadow", "k_shade", "k_probe_update",
                            "k_probe_offsets"]
    sets = [l.strip().split(": ", 1) for l in open(os.path.join(d, "sets.txt"))]
    for i, name in sets:
        ms = {}
        p = os.path.join(d, f"t{i}", "run_kernel_stats.csv")
        if os.path.exists(p):
            for r in csv.DictReader(open(p)):
                ms[short(r["Name"])] = float(r["AverageNs"]) / 1e6
        hbm = defaultdict(float)
        for sub, ctr, mult in (("f", "FETCH_SIZE", 2.0), ("w", "WRITE_SIZE", 1.0)):
            p = os.path.join(d, f"{sub}{i}", "run_counter_collection.csv")
            if not os.path.exists(p):
                continue
            vals = defaultdict(list)
            for r in csv.DictReader(open(p)):
                if r["Counter_Name"] == ctr:
                    vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
            for k, v in vals.items():
                hbm[k] += mult * sum(v) / len(v) * 1024
        cells = []
        for k in want:
            if k in ms:
                c = f"{k} {ms[k]:.4f}"
                if k in hbm:
                    c += f" ({hbm[k] / 1e9:.3f} GB)"
                cells.append(c)
        print(f"[{i}] {name}: " + " | ".join(cells))


if __name__ == "__main__":
    main()
