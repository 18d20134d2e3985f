"""The bytewise arithmetic of the sun's light-space node test (ddgi_kernels.hip
geBytes / visitNodeSun), restated in numpy and checked exhaustively on the CPU: the
unsigned compare of four packed bytes with one subtraction and one three-input boolean
function, and the gather of the eight per-child results into the 8-bit slot mask by the
high word of one multiply. The device path itself is covered by the GPU parity suite
(ARK_DDGI_SUN_BVH_LIGHT_SPACE cases), where a wrong compare would cull an occluder."""
import numpy as np

H = np.uint32(0x80808080)
L = np.uint32(0x7F7F7F7F)


def ge_bytes(x, y):
    """bit 7 of each byte: x_byte >= y_byte (geBytes: bitop3 0xb2 over x, y, d)."""
    d = ((x | H) - (y & L)).astype(np.uint32)
    return ((x & ~y) | (~(x ^ y) & d)).astype(np.uint32)


def test_ge_bytes_every_pair_every_position():
    x = np.arange(256, dtype=np.uint32).repeat(256)
    y = np.tile(np.arange(256, dtype=np.uint32), 256)
    rng = np.random.default_rng(1)
    shifts = np.array([0, 8, 16, 24], np.uint32)
    for pos in range(4):
        # the other three bytes random: no borrow may cross into or out of this byte
        bx = rng.integers(0, 256, (x.size, 4)).astype(np.uint32)
        by = rng.integers(0, 256, (x.size, 4)).astype(np.uint32)
        bx[:, pos], by[:, pos] = x, y
        X = (bx << shifts).sum(1).astype(np.uint32)
        Y = (by << shifts).sum(1).astype(np.uint32)
        got = (ge_bytes(X, Y) >> np.uint32(8 * pos + 7)) & np.uint32(1)
        assert np.array_equal(got, (x >= y).astype(np.uint32)), pos
        # every byte of the result, not only the one under test
        for other in range(4):
            g = (ge_bytes(X, Y) >> np.uint32(8 * other + 7)) & np.uint32(1)
            assert np.array_equal(g, (bx[:, other] >= by[:, other]).astype(np.uint32))


def test_slot_mask_gather_all_masks():
    for m in range(256):
        # bit 7 of byte k: child k (r0) / child k + 4 (r1), other bits cleared (& 0x80808080)
        r0 = sum(((m >> k) & 1) << (8 * k + 7) for k in range(4))
        r1 = sum(((m >> (k + 4)) & 1) << (8 * k + 7) for k in range(4))
        hi = (((r0 >> 4) | r1) * 0x20408100) >> 32
        assert hi & 0xFF == m, (m, hex(hi))


def test_clamped_bounds_only_accept_more():
    """Q clamped to [0, 255] before floor / ceil: for every plane byte and every Q of the
    old clamp range [-2, 258] the clamped test accepts whatever the unclamped one did."""
    q = np.linspace(-2.0, 258.0, 20801, dtype=np.float32)
    qc = np.clip(q, 0.0, 255.0)
    planes = np.arange(256)[:, None]
    lo_old = planes <= np.floor(q)[None, :]
    hi_old = planes >= np.ceil(q)[None, :]
    lo_new = planes <= np.floor(qc)[None, :]
    hi_new = planes >= np.ceil(qc)[None, :]
    assert not (lo_old & ~lo_new).any()
    assert not (hi_old & ~hi_new).any()
