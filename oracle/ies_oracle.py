"""CPU restatement of the IES profile -> LUT path (TEST INFRASTRUCTURE: only tests/
use it, as the checker of arkoserenderer_amd/csrc/ies_profile.cpp).

Follows IESProfile::parse (arkcore/asset/external/IESProfile.cpp:57-175),
lookupValue (:177-257), computeLookupLocation (:259-306), getValue (:308-333) and
assembleLookupTextureData (:335-352) with fp32 arithmetic (numpy float32 scalars),
ark::lerp(a, b, t) = (1 - t) a + t b (deps/arklib/include/ark/core.h:140-143).
The reference is not buildable here (ParseContext/Logging need fmt and the engine's
core), so this restatement is pinned by closed forms of the sample profiles only
(tests/test_ies.py): parity unpinned against the reference binary.
"""
from __future__ import annotations

import math
import re

import numpy as np

F = np.float32


class IesError(ValueError):
    pass


def parse(text: str) -> dict:
    lines = text.split("\n")
    if lines[0] not in ("IESNA91", "IESNA:LM-63-1995", "IESNA:LM-63-2002"):
        raise IesError("invalid version")
    i = 1
    while i < len(lines) and lines[i][:1] == "[":
        i += 1
    if i >= len(lines) or not lines[i].startswith("TILT=NONE"):
        raise IesError("only TILT=NONE")
    toks = [t for t in re.split(r"[\s,]+", "\n".join(lines[i + 1:])) if t]
    pos = 0

    def nxt(conv):
        nonlocal pos
        v = conv(toks[pos])
        pos += 1
        return v

    lamps = nxt(int)
    nxt(float)  # lumens per lamp
    mult = F(nxt(float))
    nv, nh = nxt(int), nxt(int)
    ptype, units = nxt(int), nxt(int)
    for _ in range(6):  # width, length, height, ballast, future use, input watts
        nxt(float)
    if lamps <= 0 or not mult > 0 or nv < 1 or nh < 1 or ptype not in (1, 2, 3) or units not in (1, 2):
        raise IesError("bad header")
    av = [F(nxt(float)) for _ in range(nv)]
    ah = [F(nxt(float)) for _ in range(nh)]
    for lst in (av, ah):
        if any(b <= a for a, b in zip(lst, lst[1:])):
            raise IesError("angles not increasing")
    cd = [F(mult * F(nxt(float))) for _ in range(nv * nh)]
    return {"type": ptype, "v": av, "h": ah, "cd": cd}


def _index(angle, lst):
    lo, hi = 0, len(lst) - 1
    if angle <= lst[lo]:
        return F(0)
    if angle >= lst[hi]:
        return F(hi)
    while lo < hi:
        if hi - lo == 1:
            span = F(lst[hi] - lst[lo])
            if span < F(1e-3):
                return F(lo)
            return F(F(lo) + F(F(angle - lst[lo]) / span))
        mid = (lo + hi + 1) // 2
        if angle == lst[mid]:
            return F(mid)
        if angle > lst[mid]:
            lo = mid
        else:
            hi = mid
    return F(lo)


def _lerp(a, b, t):
    return F(F(F(1) - t) * a + F(t * b))


def lookup(p: dict, angle_h, angle_v):
    angle_h, angle_v = F(angle_h), F(angle_v)
    h = angle_h
    if p["type"] == 2:
        raise IesError("type B")
    if p["type"] == 1:
        last = int(math.floor(float(p["h"][-1]) + 0.5))  # std::round, angles >= 0
        if len(p["h"]) == 1 and last == 0:
            h = F(0)
        elif last == 90:
            h = F(np.fmod(angle_h, F(90)))
            q = int(F(angle_h / F(90)))
            if q in (1, 3):
                h = F(F(90) - h)
        elif last == 180:
            h = F(np.fmod(angle_h, F(180)))
            if angle_h >= F(180):
                h = F(F(360) - angle_h)
        elif 180 < last <= 360:
            h = angle_h
        else:
            raise IesError("last horizontal angle")
    lh, lv = _index(h, p["h"]), _index(angle_v, p["v"])
    nh, nv = len(p["h"]), len(p["v"])

    def at(x, y):
        x = max(0, min(x, nh - 1))
        y = max(0, min(y, nv - 1))
        return p["cd"][y + nv * x]

    x, y = int(lh), int(lv)
    dx, dy = F(lh - F(x)), F(lv - F(y))
    top = _lerp(at(x, y + 1), at(x + 1, y + 1), dx)
    bot = _lerp(at(x, y), at(x + 1, y), dx)
    return _lerp(bot, top, dy)


def lut(text: str, size: int = 256) -> np.ndarray:
    p = parse(text)
    out = np.empty((size, size), np.float32)
    for y in range(size):
        horizontal = F(F(F(y) / F(size)) * F(360))
        for x in range(size):
            vertical = F(F(F(x) / F(size)) * F(180))
            out[y, x] = lookup(p, horizontal, vertical)
    return out
