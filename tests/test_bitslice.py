"""The SWAR bit transpose of bitslice.h (tr8) as the device code computes it:
block swaps paired so that two dwords are shifted by ONE 64-bit shift, the
bits crossing the dword boundary discarded by the select masks.  Checked
against the definition of the bit-plane layout (plane a, byte q, bit w =
bit a of byte 4w + q of the lane's 32 bytes) on random lanes, and for being
its own inverse.  The device instructions themselves are covered by every
GPU parity test (tests/test_gpu_*.py) and by tools/tr8_codegen.sh."""
import numpy as np

M32 = np.uint64(0xFFFFFFFF)
MASKS = {4: 0x0F0F0F0F, 2: 0x33333333, 1: 0x55555555}


def swap_blk2(W, lo0, lo1, hi0, hi1, s):
    """bitslice.h swap_blk2<s>: v_lshrrev_b64 of (lo1:lo0), v_lshlrev_b64 of
    (hi1:hi0), four v_bitop3 0xE4 selects."""
    m = np.uint64(MASKS[s])
    nm = ~m & M32
    sh = np.uint64(s)
    lpair = ((W[lo1] << np.uint64(32)) | W[lo0]) >> sh
    hpair = (((W[hi1] << np.uint64(32)) | W[hi0]) << sh) & np.uint64(0xFFFFFFFFFFFFFFFF)
    l0, l1 = lpair & M32, lpair >> np.uint64(32)
    h0, h1 = hpair & M32, hpair >> np.uint64(32)
    n_lo0 = (W[lo0] & m) | (h0 & nm)
    n_lo1 = (W[lo1] & m) | (h1 & nm)
    n_hi0 = (l0 & m) | (W[hi0] & nm)
    n_hi1 = (l1 & m) | (W[hi1] & nm)
    W[lo0], W[lo1], W[hi0], W[hi1] = n_lo0, n_lo1, n_hi0, n_hi1


def tr8(W):
    W = [w.copy() for w in W]
    swap_blk2(W, 0, 1, 4, 5, 4)
    swap_blk2(W, 2, 3, 6, 7, 4)
    swap_blk2(W, 0, 1, 2, 3, 2)
    swap_blk2(W, 4, 5, 6, 7, 2)
    swap_blk2(W, 0, 2, 1, 3, 1)
    swap_blk2(W, 4, 6, 5, 7, 1)
    return W


def planes_by_definition(seg):
    """seg: [n][32] bytes -> [8][n] dwords, plane a byte q bit w = bit a of
    byte 4w + q."""
    n = seg.shape[0]
    out = np.zeros((8, n), np.uint64)
    for a in range(8):
        for q in range(4):
            for w in range(8):
                bit = (seg[:, 4 * w + q] >> a) & 1
                out[a] |= bit.astype(np.uint64) << np.uint64(8 * q + w)
    return out


def test_tr8_matches_plane_definition_and_is_self_inverse():
    rng = np.random.default_rng(7)
    seg = rng.integers(0, 256, size=(4096, 32), dtype=np.uint8)
    # W[w] = bytes 4w .. 4w+3, little endian (as the lane loads them)
    W = [seg[:, 4 * w:4 * w + 4].copy().view(np.uint32)[:, 0].astype(np.uint64) for w in range(8)]
    P = tr8(W)
    ref = planes_by_definition(seg)
    for a in range(8):
        assert np.array_equal(P[a], ref[a])
    back = tr8(P)
    for w in range(8):
        assert np.array_equal(back[w], W[w])


def test_boundary_bits_never_selected():
    """The s bits a 64-bit shift moves across the dword boundary sit where
    the select mask takes the other operand."""
    for s, m in MASKS.items():
        top = ((1 << s) - 1) << (32 - s)     # lo0 >> s receives lo1's low bits here
        bottom = (1 << s) - 1                 # hi1 << s receives hi0's high bits here
        assert m & top == 0
        assert (~m & 0xFFFFFFFF) & bottom == 0

