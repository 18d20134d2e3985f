"""Host restatement of the windowed Z-slab exchange's packet layout (test
infrastructure; the device path is ddgi_exchange.hip behind ark_ddgi_pack_window /
ark_ddgi_unpack_window). A window (first, K) of an N-probe grid; rank q of P owns the
probes with z in [q Z/P, (q+1) Z/P) (probe index order x, then z, then y:
ddgi/common.glsl:36-51). Its packets are its window probes in window order (the slot
order slabRankOf gives), each the probe's 10 x 10 irradiance tile (RGBA16F, border
included, row by row) then its 18 x 18 visibility tile (RG16F); every rank's region is
padded to the largest slab share."""
from types import SimpleNamespace

import numpy as np

PACKET_BYTES = 10 * 10 * 8 + 18 * 18 * 4  # ARK_DDGI_WINDOW_PACKET_BYTES
TI, TV = 10, 18


def window_probes(dims, first, K):
    X, Y, Z = dims
    N = X * Y * Z
    return (first + np.arange(K, dtype=np.int64)) % N


def slab_lists(dims, P, first, K):
    """Each rank's window probes in slot order."""
    X, Y, Z = dims
    p = window_probes(dims, first, K)
    owner = ((p % (X * Z)) // X) // (Z // P)
    return [p[owner == q] for q in range(P)]


def info(dims, P, rank, first, K):
    """ark_ddgi_window_exchange_info's fields."""
    X, Y, Z = dims
    lists = slab_lists(dims, P, first, K)
    full = K == X * Y * Z
    per = max(len(v) for v in lists)
    return SimpleNamespace(full_bands=int(full), probes_per_rank=per, my_probes=len(lists[rank]), first_probe=first, probe_updates=K,
                           bytes_per_rank=0 if full else per * PACKET_BYTES)


def _tile(dims, p, t):
    X, Y, Z = dims
    y, rem = divmod(int(p), X * Z)
    z, x = divmod(rem, X)
    return z * t, (x + y * X) * t


def pack(irr, vis, dims, P, rank, first, K):
    """This rank's region (bytes_per_rank). irr: (H_i, W_i * 4) uint16; vis: (H_v, W_v * 2) uint16."""
    w = info(dims, P, rank, first, K)
    out = np.zeros(w.bytes_per_rank, np.uint8)
    for s, p in enumerate(slab_lists(dims, P, first, K)[rank]):
        r0, c0 = _tile(dims, p, TI)
        a = irr[r0:r0 + TI, c0 * 4:(c0 + TI) * 4]
        r1, c1 = _tile(dims, p, TV)
        b = vis[r1:r1 + TV, c1 * 2:(c1 + TV) * 2]
        out[s * PACKET_BYTES:(s + 1) * PACKET_BYTES] = np.concatenate([np.ascontiguousarray(a).view(np.uint8).ravel(),
                                                                     np.ascontiguousarray(b).view(np.uint8).ravel()])
    return out


def unpack(irr, vis, buf, dims, P, rank, first, K):
    """Writes every other rank's packets (buf: P regions) into their tiles, in place."""
    w = info(dims, P, rank, first, K)
    n = w.bytes_per_rank
    for q, probes in enumerate(slab_lists(dims, P, first, K)):
        if q == rank:
            continue
        for s, p in enumerate(probes):
            pkt = buf[q * n + s * PACKET_BYTES:q * n + (s + 1) * PACKET_BYTES]
            r0, c0 = _tile(dims, p, TI)
            irr[r0:r0 + TI, c0 * 4:(c0 + TI) * 4] = pkt[:TI * TI * 8].view(np.uint16).reshape(TI, TI * 4)
            r1, c1 = _tile(dims, p, TV)
            vis[r1:r1 + TV, c1 * 2:(c1 + TV) * 2] = pkt[TI * TI * 8:].view(np.uint16).reshape(TV, TV * 2)
