"""The bytewise arithmetic of the sun's light-space node test (ddgi_kernels.hip
visitNodeSun), restated in numpy and checked exhaustively on the CPU: with 7-bit planes
(Bvh8CollapseOptions::quant_max = 127) and the query clamped to [0, 127], one 32-bit
subtraction compares four packed bytes ((x | 0x80) - y: bit 7 of each byte says
x >= y), and the high word of one multiply gathers the eight per-child results into
the 8-bit slot mask. The device path itself is covered by the GPU parity suite
(ARK_SUN_BVH=1 cases), where a wrong compare would cull an occluder; the 7-bit planes
of the BVH the library builds by tests/test_sun_bvh.py (ark_ddgi_debug_sun_bvh_check
returns 3 for a plane above 127)."""
import numpy as np

H = np.uint32(0x80808080)


def ge_bytes7(x, y):
    """bit 7 of each byte: x_byte >= y_byte, for bytes <= 127."""
    return (((x | H) - y).astype(np.uint32)) & H


def test_ge_bytes7_every_pair_every_position():
    x = np.arange(128, dtype=np.uint32).repeat(128)
    y = np.tile(np.arange(128, dtype=np.uint32), 128)
    rng = np.random.default_rng(1)
    shifts = np.array([0, 8, 16, 24], np.uint32)
    for pos in range(4):
        # the other three bytes random: no borrow may cross into or out of this byte
        bx = rng.integers(0, 128, (x.size, 4)).astype(np.uint32)
        by = rng.integers(0, 128, (x.size, 4)).astype(np.uint32)
        bx[:, pos], by[:, pos] = x, y
        X = (bx << shifts).sum(1).astype(np.uint32)
        Y = (by << shifts).sum(1).astype(np.uint32)
        g = ge_bytes7(X, Y)
        for other in range(4):
            got = (g >> np.uint32(8 * other + 7)) & np.uint32(1)
            assert np.array_equal(got, (bx[:, other] >= by[:, other]).astype(np.uint32)), (pos, other)


def test_slot_mask_gather_all_masks():
    for m in range(256):
        # bit 7 of byte k: child k (r0) / child k + 4 (r1), other bits cleared (& 0x80808080)
        r0 = sum(((m >> k) & 1) << (8 * k + 7) for k in range(4))
        r1 = sum(((m >> (k + 4)) & 1) << (8 * k + 7) for k in range(4))
        hi = (((r0 >> 4) | r1) * 0x20408100) >> 32
        assert hi & 0xFF == m, (m, hex(hi))


def test_clamped_bounds_only_accept_more():
    """Q clamped to [0, 127] before floor / ceil: for every 7-bit plane and every Q of a
    wide range the clamped test accepts whatever the unclamped one did."""
    q = np.linspace(-4.0, 131.0, 13501, dtype=np.float32)
    qc = np.clip(q, 0.0, 127.0)
    planes = np.arange(128)[:, None]
    lo_old = planes <= np.floor(q)[None, :]
    hi_old = planes >= np.ceil(q)[None, :]
    lo_new = planes <= np.floor(qc)[None, :]
    hi_new = planes >= np.ceil(qc)[None, :]
    assert not (lo_old & ~lo_new).any()
    assert not (hi_old & ~hi_new).any()

