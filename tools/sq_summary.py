"""Summarises a tools/prof_sq.sh output directory: per kernel, SQ/TCC counters
summed over its dispatches and the derived ratios (per-wave fractions of
SQ_WAVE_CYCLES, VALU issue per SIMD-quad-cycle, L2 hit rate).

    python tools/sq_summary.py gpurun_out/<tag> [<tag> --json [--latest]] [> profiles/<tag>_sq.txt]

--json writes profiles/<tag>_sq.json (per kernel ratios + the library hash of the
profiled bench run); --latest also copies it to profiles/latest_sq.json, which
bench.py reads when the hash matches its own library.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = name.split("(")[0].replace("void ", "").replace("ark::dev::", "")
    return name


def base_name(name):
    """k_trace<false, 6> -> k_trace (timed variants only; counting ones are skipped)."""
    m = re.match(r"(k_[a-z0-9_]+)(<([a-z]+)[^>]*>)?", name)
    if not m or m.group(3) == "true":
        return None
    if m.group(1) == "k_trace_shadow" and m.group(2):
        mode = m.group(2).rstrip(">").split(",")[-1].strip()
        # <.., .., MODE>: 1 the sun's light-space traversal, 2 the sun's then the other lights'
        return {"1": "k_trace_shadow_sun", "2": "k_trace_shadow_sunw"}.get(mode, m.group(1))
    return m.group(1)


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
    if "--json" in sys.argv:
        tag = sys.argv[2]
        lib_sha, launches = None, {}
        for line in open(os.path.join(d, "sq1.log")):
            if line.startswith("{"):
                try:
                    lib_sha = json.loads(line)["config"].get("lib_sha16")
                except (ValueError, KeyError):
                    pass
        calls = collections.Counter()
        for r in csv.DictReader(open(glob.glob(f"{d}/sq1/run_counter_collection.csv")[0])):
            if r["Counter_Name"] == "SQ_WAVES":
                calls[short(r["Kernel_Name"])] += 1
        # effective clock per kernel (MI355X_MICROARCH.md, DVFS give-back): GRBM_GUI_ACTIVE
        # summed over the 8 XCDs / 8 / the dispatch's wall time, from the tcc pass
        grbm, wall = collections.defaultdict(float), collections.defaultdict(float)
        for f in glob.glob(f"{d}/tcc/run_counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                    k = short(r["Kernel_Name"])
                    grbm[k] += float(r["Counter_Value"])
                    wall[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        kernels = {}
        for k, v in agg.items():
            b = base_name(k)
            wc = v.get("SQ_WAVE_CYCLES", 0)
            if b is None or wc <= 0:
                continue
            hit, miss = v.get("TCC_HIT_sum", 0.0), v.get("TCC_MISS_sum", 0.0)
            n = max(1, calls[k])
            kernels[b] = {"valu_active_per_wave": round(v.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3),
                          "wait_inst_any_per_wave": round(v.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
                          "wait_any_per_wave": round(v.get("SQ_WAIT_ANY", 0) / wc, 3),
                          "valu_insts_per_launch": round(v.get("SQ_INSTS_VALU", 0) / n),
                          "salu_insts_per_launch": round(v.get("SQ_INSTS_SALU", 0) / n),
                          "vmem_rd_insts_per_launch": round(v.get("SQ_INSTS_VMEM_RD", 0) / n),
                          "l2_hit": round(hit / (hit + miss), 3) if hit + miss else None,
                          "clock_ghz_effective": round(grbm[k] / 8 / wall[k] / 1e9, 3) if wall[k] > 0 else None}
        out = {"tag": tag, "lib_sha16": lib_sha, "source": f"rocprofv3 --pmc SQ_*/TCC_* passes (tools/prof_sq.sh), profiles/{tag}_sq.*",
               "kernels": kernels}
        with open(os.path.join(ROOT, "profiles", f"{tag}_sq.json"), "w") as fh:
            json.dump(out, fh, indent=1)
        if "--latest" in sys.argv:
            with open(os.path.join(ROOT, "profiles", "latest_sq.json"), "w") as fh:
                json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
