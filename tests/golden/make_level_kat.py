"""Generates tests/golden/level_kat.json: the reference's own math library
(deps/arklib, header-only, compiled here as oracle/_ref/level_kat by
oracle/Makefile.ref) evaluated on the transforms and light colours of the in-tree
level fixtures (tests/assets/levels/*.arklvl) plus synthetic cases. Inputs and
outputs are float32 bit patterns. Run where /root/reference exists:
    make -C oracle -f Makefile.ref && python tests/golden/make_level_kat.py
"""
import glob
import json
import os
import struct
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def hx(v):
    return "%08x" % struct.unpack("<I", struct.pack("<f", float(np.float32(v))))[0]


def main():
    transforms, colors = [], []
    for f in sorted(glob.glob(os.path.join(ROOT, "tests", "assets", "levels", "*.arklvl"))):
        L = json.load(open(f))["level"]
        for item in L.get("objects", []) + L.get("lights", []):
            tr = item["transform"]
            t, q, s = tr["translation"], tr["orientation"], tr["scale"]
            transforms.append([t["x"], t["y"], t["z"], q["x"], q["y"], q["z"], q["w"], s["x"], s["y"], s["z"]])
        for la in L.get("lights", []):
            c = la["color"]
            colors.append([c["x"], c["y"], c["z"]])
    rng = np.random.default_rng(20261016)
    for _ in range(24):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        transforms.append(list(rng.uniform(-10, 10, 3)) + list(q) + list(rng.uniform(0.01, 3, 3)))
    for _ in range(24):
        colors.append(list(rng.uniform(0, 1, 3)))
    colors.append([0.04045, 0.0404, 0.0405])
    colors.append([0.0, 1.0, 0.5])
    lines = ["T " + " ".join(hx(v) for v in t) for t in transforms] + ["C " + " ".join(hx(v) for v in c) for c in colors]
    exe = os.path.join(ROOT, "oracle", "_ref", "level_kat")
    out = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True).stdout.split("\n")
    rec = {"source": "oracle/_ref/level_kat (deps/arklib quaternion.h / transform.h / color.h)", "transforms": [], "colors": []}
    for inp, o in zip(lines, out):
        w = o.split()
        if inp[0] == "T":
            rec["transforms"].append({"in": inp.split()[1:], "forward": w[1:4], "right": w[4:7], "up": w[7:10], "matrix_colmajor": w[10:26]})
        else:
            rec["colors"].append({"in": inp.split()[1:], "linear": w[1:4]})
    with open(os.path.join(ROOT, "tests", "golden", "level_kat.json"), "w") as fh:
        json.dump(rec, fh)
    print(f"{len(rec['transforms'])} transforms, {len(rec['colors'])} colours")


if __name__ == "__main__":
    main()
