"""Summarises a tools/prof_sq.sh output directory: per kernel, SQ/TCC counters
summed over its dispatches and the derived ratios (per-wave fractions of
SQ_WAVE_CYCLES, VALU issue per SIMD-quad-cycle, L2 hit rate).

    python tools/sq_summary.py gpurun_out/<tag> [> profiles/<tag>_sq.txt]
"""
import collections
import csv
import glob
import sys


def short(name):
    name = name.split("(")[0].replace("void ", "").replace("ark::dev::", "")
    return name


def main():
    d = sys.argv[1]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for sub in ("sq1", "sq2", "tcc"):
        for f in glob.glob(f"{d}/{sub}/run_counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                agg[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        if v.get("SQ_WAVE_CYCLES", 0) <= 0:
            continue
        wc = v["SQ_WAVE_CYCLES"]
        hit = v.get("TCC_HIT_sum", 0.0)
        miss = v.get("TCC_MISS_sum", 0.0)
        print(f"{k}")
        print("   waves %.3g  wave-cycles %.3g  busy-cycles %.3g" % (v.get("SQ_WAVES", 0), wc, v.get("SQ_BUSY_CYCLES", 0)))
        print("   per wave: wait_any %.2f  wait_inst_any %.2f  active_inst_any %.2f  active_valu %.2f  active_lds %.3f" % (
            v.get("SQ_WAIT_ANY", 0) / wc, v.get("SQ_WAIT_INST_ANY", 0) / wc, v.get("SQ_ACTIVE_INST_ANY", 0) / wc,
            v.get("SQ_ACTIVE_INST_VALU", 0) / wc, v.get("SQ_ACTIVE_INST_LDS", 0) / wc))
        print("   insts: valu %.3g  salu %.3g  vmem_rd %.3g  lds %.3g   L2 hit %.3f  TCP accesses %.3g" % (
            v.get("SQ_INSTS_VALU", 0), v.get("SQ_INSTS_SALU", 0), v.get("SQ_INSTS_VMEM_RD", 0), v.get("SQ_INSTS_LDS", 0),
            hit / (hit + miss) if hit + miss else 0.0, v.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0)))


if __name__ == "__main__":
    main()
