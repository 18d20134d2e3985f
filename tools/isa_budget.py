"""Instruction budget of a kernel in device assembly (hipcc --cuda-device-only -S):
per basic block the VALU / SALU / vector-memory / LDS instruction counts, the
kernel's register use and spills, and the loop blocks of the traversal step.

    python tools/isa_budget.py <file.s> [kernel-substring] [--blocks] [--json]

Build the assembly with the library's own flags (tools/isa_budget.py --build OUT.s
[EXTRA...] runs hipcc on ddgi_kernels.hip with the Makefile's kernel flags plus EXTRA).
"""
import json
import re
import subprocess
import sys
from collections import Counter, OrderedDict

ROOT = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
FLAGS = ["-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wno-unused-function",
         "-munsafe-fp-atomics", "-fno-slp-vectorize", "-mllvm", "-amdgpu-set-wave-priority", "--cuda-device-only", "-S"]


def kind(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def parse(path, key):
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\w*:", l) and key in l]
    if not starts:
        raise SystemExit(f"no kernel matching {key}")
    i0 = starts[0]
    name = lines[i0].split(":")[0]
    i1 = next(i for i in range(i0, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = []
    for l in lines[i0 + 1:i1]:
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            continue
        s = l.strip()
        if s and not s.startswith((".", ";")):
            blocks[cur].append(s.split()[0])
    meta = {}
    text = "\n".join(lines)
    m = re.search(r"\.name:\s+" + re.escape(name) + r"\n", text)
    if m:
        # the entry's scalar fields follow its .name up to .wavefront_size
        tail = text[m.end():m.end() + 4000]
        tail = tail[:tail.find(".wavefront_size")] if ".wavefront_size" in tail else tail
        for k in ("sgpr_count", "vgpr_count", "vgpr_spill_count", "sgpr_spill_count", "group_segment_fixed_size", "private_segment_fixed_size"):
            mm = re.search(r"\." + k + r":\s+(\d+)", tail)
            if mm:
                meta[k] = int(mm.group(1))
    return name, blocks, meta


def main():
    if sys.argv[1] == "--build":
        out, extra = sys.argv[2], sys.argv[3:]
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-o", out, "ddgi_kernels.hip"], cwd=f"{ROOT}/arkoserenderer_amd/csrc", check=True,
                       stderr=subprocess.DEVNULL)
        return
    path = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "k_traceILb0ELi6ENS0_9ProbeRays"
    name, blocks, meta = parse(path, key)
    tot = Counter()
    rows = []
    for b, ops in blocks.items():
        c = Counter(kind(o) for o in ops)
        tot += c
        rows.append((b, len(ops), dict(c), Counter(ops).most_common(6)))
    out = {"kernel": name, "meta": meta, "total": dict(tot), "blocks": {b: c for b, _, c, _ in rows}}
    if "--json" in sys.argv:
        print(json.dumps(out))
        return
    print(name)
    print("registers:", meta)
    print("static totals:", dict(tot))
    if "--blocks" in sys.argv:
        for b, n, c, top in rows:
            print(f"{b:12s} {n:4d} {c} {top}")


if __name__ == "__main__":
    main()
