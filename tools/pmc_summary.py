"""Summarises a tools/prof_run.sh output directory into profiles/.

Per kernel: average duration (kernel-trace stats) and HBM traffic per launch from
the PMC passes. Units/corrections per MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE reads 1/2 of the bytes of a wide
coalesced streaming read, so the corrected read bytes are 2 x FETCH_SIZE x 1024
(the guide's prescription; uncalibrated for our 16-B gather pattern, so both the
raw and the corrected figure are kept). WRITE_SIZE x 1024 as is.

    python tools/pmc_summary.py gpurun_out/<tag> <tag> [--latest]
"""
import csv
import re
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    """ark::dev::k_trace<false, 6, ProbeRays>(...) -> k_trace; <true, ...> -> k_trace_counting;
    the reflections' instantiations -> k_refl_trace / k_refl_shadow_gen; the sun's
    shadow traversal k_trace_shadow<.., .., true> -> k_trace_shadow_sun."""
    m = re.search(r"\b(k_[a-z0-9_]+)(<([a-z]+)[^>]*>)?", name)
    if not m:
        return name
    base = m.group(1)
    if base == "k_trace_shadow" and m.group(2):
        mode = m.group(2).rstrip(">").split(",")[-1].strip()
        # <COUNT, WPE, MODE>: 1 the sun's light-space traversal, 2 the sun's then the other lights'
        base = {"1": "k_trace_shadow_sun", "2": "k_trace_shadow_sunw"}.get(mode, base)
    if base == "k_trace" and "ListRays" in name:
        return "k_refl_trace"
    if base == "k_shadow_gen":
        return "k_refl_shadow_gen" if m.group(3) == "true" else base
    return base + "_counting" if m.group(3) == "true" else base


def main():
    src, tag = sys.argv[1], sys.argv[2]
    latest = "--latest" in sys.argv
    stats = {}
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as fh:
        for r in csv.DictReader(fh):
            stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                       "pct": float(r["Percentage"])}
    pmc = defaultdict(lambda: defaultdict(list))
    pmc_ms = defaultdict(list)
    for sub in ("fetch", "write"):
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        with open(p) as fh:
            rows = sorted(csv.DictReader(fh), key=lambda r: int(r["Dispatch_Id"]))
        refl = False  # the RT reflections' launches share the shadow traversal kernel
        for r in rows:
            k = short(r["Kernel_Name"])
            refl = refl or k == "k_refl_setup"
            if refl and k == "k_trace_shadow":
                k = "k_refl_trace_shadow"
            pmc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if sub == "fetch":
                pmc_ms[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    # kernels the (probe-path-only) trace pass did not run: the consumers of the byte
    # passes, timed by the PMC pass's own timestamps
    for k, v in pmc_ms.items():
        if k not in stats and k.startswith(("k_refl", "k_lighting")):
            stats[k] = {"calls": len(v), "avg_ms": sum(v) / len(v), "avg_ms_source": "PMC pass dispatch timestamps"}
    kernels = {}
    for k, st in stats.items():
        e = dict(st)
        c = pmc.get(k, {})
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            f = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
            w = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
            e["fetch_kib_raw"] = round(f, 1)
            e["write_kib"] = round(w, 1)
            e["hbm_bytes_per_launch"] = int((2.0 * f + w) * 1024)
            e["hbm_bytes_per_launch_uncorrected"] = int((f + w) * 1024)
            e["hbm_gbs"] = round(e["hbm_bytes_per_launch"] / (st["avg_ms"] * 1e-3) / 1e9, 1)
        kernels[k] = e
    cfg = {}
    log = os.path.join(src, "trace.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{"):
                try:
                    j = json.loads(line)
                    cfg = {"triangles": j["config"]["triangles"], "grid": j["config"]["grid"],
                           "rays_per_probe": j["config"]["rays_per_probe"], "lib_sha16": j["config"].get("lib_sha16"), "bench": j}
                except Exception:
                    pass
    out = {"tag": tag, "source": f"rocprofv3 --kernel-trace --stats + --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), profiles/{tag}_*",
           "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md §HBM gfx950 FETCH_SIZE halving)",
           "config": cfg, "kernels": kernels}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", f"{tag}_summary.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    for sub in ("fetch", "write"):
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if os.path.exists(p):
            shutil.copy(p, os.path.join(ROOT, "profiles", f"{tag}_pmc_{sub}.csv"))
    if latest:
        with open(os.path.join(ROOT, "profiles", "latest_pmc.json"), "w") as fh:
            json.dump(out, fh, indent=1)
    for k, e in kernels.items():
        print(k, e)


if __name__ == "__main__":
    main()
