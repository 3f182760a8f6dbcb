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


def _run_asm(lines, regs, lds, addr):
    """Interpret the few instruction forms gen_tc_handlers.py's transposes
    use: 64-bit shifts, v_bitop3 0xE4, v_mov of a literal, ds_read_b128 /
    ds_write_b128 at %0 + offset, s_waitcnt lgkmcnt(n), s_nop.  LDS reads land
    only when a wait covers them (in issue order, as the hardware counts), so
    a register read before its wait sees the stale value and fails the test."""
    import re
    pending = []  # [kind, payload] in issue order (reads and writes)

    def reg(tok):
        return int(re.match(r"v\[?(\d+)", tok).group(1))

    for ln in lines:
        op, _, rest = ln.partition(" ")
        args = [a.strip() for a in rest.split(",")] if rest else []
        if op == "s_nop":
            continue
        if op == "s_waitcnt":
            n = int(re.search(r"lgkmcnt\((\d+)\)", ln).group(1))
            while len(pending) > n:
                kind, p = pending.pop(0)
                if kind == "r":
                    base, off = p
                    for i in range(4):
                        regs[base + i] = lds.get(addr + off + 4 * i, 0)
            continue
        if op == "v_mov_b32":
            regs[reg(args[0])] = int(args[1], 16)
        elif op in ("v_lshrrev_b64", "v_lshlrev_b64"):
            d, s, src = reg(args[0]), int(args[1]), reg(args[2])
            v = regs[src] | (regs[src + 1] << 32)
            v = (v >> s) if op == "v_lshrrev_b64" else ((v << s) & 0xFFFFFFFFFFFFFFFF)
            regs[d], regs[d + 1] = v & 0xFFFFFFFF, v >> 32
        elif op == "v_bitop3_b32":
            assert "bitop3:0xe4" in ln
            d, a, c, m = (reg(x) for x in args[:4])
            regs[d] = (regs[a] & regs[m]) | (regs[c] & ~regs[m] & 0xFFFFFFFF)
        elif op == "ds_read_b128":
            off = int(re.search(r"offset:(\d+)", ln).group(1))
            pending.append(["r", (reg(args[0]), off)])
        elif op == "ds_write_b128":
            off = int(re.search(r"offset:(\d+)", ln).group(1))
            base = reg(args[1])
            for i in range(4):  # data read at issue, stored in order
                lds[addr + off + 4 * i] = regs[base + i]
            pending.append(["w", None])
        else:
            raise AssertionError("unexpected instruction " + ln)
    assert all(k == "w" for k, _ in pending), "a read left outstanding"


def test_jitw_asm_transposes_match_tr8():
    """gen_tc_handlers.py RSGPU_JW_TR{n}_NV{nv}: k_rs_jitw's per-chunk source
    transposes in hand-allocated registers (every 64-bit shift on an
    even-aligned pair, no moves), the first two sources read together and the
    third while the second is transposed.  Interpreted on random lanes: every
    source's 32 bytes in LDS become exactly bitslice.h tr8's planes, at their
    own offsets, for n = 1..3 sources and both wave strides."""
    import os
    import random
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "storage-benchmarks_amd", "csrc"))
    import gen_tc_handlers as g
    rng = random.Random(3)
    for nv in (2, 4):
        stride = nv * 2048
        for n in (1, 2, 3):
            lines = g.jw_transposes(n, stride)
            for _ in range(40):
                lds, addr, want = {}, 16 * rng.randrange(64), {}
                for i in range(n):
                    seg = [rng.randrange(256) for _ in range(32)]
                    W = [np.uint64(int.from_bytes(bytes(seg[4 * w:4 * w + 4]), "little")) for w in range(8)]
                    P = tr8([np.array([w]) for w in W])
                    for w in range(8):
                        off = i * stride + (w // 4) * 1024 + 4 * (w % 4)
                        lds[addr + off] = int(W[w])
                        want[addr + off] = int(P[w][0])
                regs = {r: rng.randrange(1 << 32) for r in range(0, 64)}
                _run_asm(lines, regs, lds, addr)
                for k, v in want.items():
                    assert lds[k] == v, (nv, n, k)
            regs_used = {int(x) for ln in lines for x in __import__("re").findall(r"v\[?(\d+)", ln)}
            assert min(regs_used) >= 10 and max(regs_used) <= 36  # RSGPU_JW_TR_CLOBBERS
