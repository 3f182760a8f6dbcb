#!/usr/bin/env python3
"""Generate tc_handlers.inc: the 256 threaded-code handlers of k_rs_tc.

Handler c applies "acc ^= c * x" to one bit-sliced accumulator (8 planes of
32 bytes per lane, rs_bitsliced.hip) from the four-Russians tables of x:
    acc_b ^= L[m_b & 15] ^ H[m_b >> 4],   m_b = row b of c's 8x8 GF(2) matrix
one v_bitop3 (or v_xor_b32_e64 when one table index is 0) per plane, then
returns with s_setpc_b64.  Every handler is exactly STRIDE bytes so that the
address of handler c is base + c * STRIDE.

Register contract (must match rs_tc.hip; the kernel limits the compiler to
v0..v63 with amdgpu_num_vgpr(64), so v64..v127 belong to the asm alone):
    acc slot 0 planes   v[ACC .. ACC+7]  (slot s is reached with
                        s_set_gpr_idx_on 8*s, gpr_idx(SRC0,DST))
    L[n], H[n], n = 1..15   v[reg_l(n)], v[reg_h(n)] (layouts below)
    return address      s[RET:RET+1]
    address banks       s[64:79], s[84:99]; m0 save s63; chain continuation s[80:81]; planes v[24:31]
    (all of these are clobbers of the one asm statement per chunk)

usage: gen_tc_handlers.py OUT.inc
"""
import os
import sys

ACC = 64
RET = 82
STRIDE = 72  # 8 x 8-byte VOP3 + s_setpc_b64 (4) + s_nop pad (4)

# Table registers.  "late" layout (default): the 8 single-plane entries
# L1 L2 L4 L8 H1 H2 H4 H8 are v24..v31, so the next source's planes are read
# from LDS straight into them (after the current source's dispatch; no
# staging copies); the 11 composite L entries follow at v32.., then the 11 H.
# "staged" layout (RSGPU_TC_LAYOUT=staged): L[n] = v[31 + n], H[n] = v[46 + n],
# planes read one source ahead into v24..v31 and copied in (8 v_mov).
LAYOUT = os.environ.get("RSGPU_TC_LAYOUT", "late")
assert LAYOUT in ("late", "staged"), LAYOUT
_COMPOSITE = [n for n in range(1, 16) if n & (n - 1)]


def reg_l(n: int) -> int:
    if LAYOUT == "staged":
        return 31 + n
    return 24 + (n.bit_length() - 1) if n & (n - 1) == 0 else 32 + _COMPOSITE.index(n)


def reg_h(n: int) -> int:
    if LAYOUT == "staged":
        return 46 + n
    return 28 + (n.bit_length() - 1) if n & (n - 1) == 0 else 43 + _COMPOSITE.index(n)


TABLE_REGS = sorted({reg_l(n) for n in range(1, 16)} | {reg_h(n) for n in range(1, 16)})


def gf_mul(a: int, b: int) -> int:
    """GF(2^8) product, polynomial 0x11D (isa/ec_base.c gf_mul)."""
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = ((a << 1) ^ (0x11D if a & 0x80 else 0)) & 0xFF
        b >>= 1
    return r


def mat_row(c: int, b: int) -> int:
    """Row b of the matrix of x -> c*x: bit a set iff bit b of c*2^a is set."""
    row = 0
    for a in range(8):
        if (gf_mul(c, 1 << a) >> b) & 1:
            row |= 1 << a
    return row


# Chained dispatch.  RSGPU_TC_CHAIN = number of handler copies (default 3):
# copy k works on v[ACC + 8k ..] and, except the last copy, continues at the
# address the chunk put in s[RA_LIST[k]] (the next slot's handler) instead of
# returning; the last copy returns.  With GPR indexing relocating a whole
# group by one index, a group of slots costs one s_swappc, one jump per
# further slot and one return.  1 = call/return per slot; 2 = slot pairs
# (3 jumps, 5 SALU per pair); 3 = triples (slots 0-2, 3-5 and 6-7).  A group
# at index 0 runs before index mode is switched on: GPR index mode costs
# every VALU instruction it covers about one issue cycle
# (tools/ubench_idx.hip), and these slots need no relocation.
CHAIN = int(os.environ.get("RSGPU_TC_CHAIN", "3") or "1")
CHAIN = 1 if CHAIN == 0 else CHAIN
assert CHAIN in (1, 2, 3, 4), CHAIN
NCOPY = CHAIN
NHANDLERS = 256 * NCOPY
RA_LIST = [80, 60, 58][: NCOPY - 1]  # s[80:81], s[60:61], s[58:59]; s[100:101] is reserved on gfx950
# dispatch groups: (first slot, handler copy of each slot, GPR index)
if NCOPY == 1:
    GROUPS = [(sl, [0], 8 * sl) for sl in range(8)]
elif NCOPY == 2:
    GROUPS = [(2 * p, [0, 1], 16 * p) for p in range(4)]
elif NCOPY == 3:
    GROUPS = [(0, [0, 1, 2], 0), (3, [0, 1, 2], 24), (6, [1, 2], 40)]
else:  # 4: quads (72 KB of handlers; an instruction-cache experiment)
    GROUPS = [(0, [0, 1, 2, 3], 0), (4, [0, 1, 2, 3], 32)]
SLOT_COPY = [0] * 8
for _s0, _ks, _ix in GROUPS:
    assert _ks[-1] == NCOPY - 1  # a group ends with the returning copy
    for _i, _k in enumerate(_ks):
        SLOT_COPY[_s0 + _i] = _k
        assert 8 * (_s0 + _i) == 8 * _k + _ix  # one index relocates the group
RA = RA_LIST[0] if RA_LIST else None


def handler(c: int, copy: int = 0) -> list:
    """Handler of coefficient c, handler copy `copy` (chained dispatch)."""
    copy = int(copy)
    ret = RA_LIST[copy] if copy < NCOPY - 1 else RET
    base = ACC + 8 * copy
    if c == 0:
        # no-op: continue at once; pad to STRIDE with never-executed s_nop
        return [f"s_setpc_b64 s[{ret}:{ret + 1}]"] + ["s_nop 0"] * ((STRIDE - 4) // 4)
    ins = []
    for b in range(8):
        m = mat_row(c, b)
        lo, hi = m & 15, m >> 4
        acc = base + b
        if lo and hi:
            ins.append(f"v_bitop3_b32 v{acc}, v{acc}, v{reg_l(lo)}, v{reg_h(hi)} bitop3:0x96")
        elif lo:
            ins.append(f"v_xor_b32_e64 v{acc}, v{acc}, v{reg_l(lo)}")
        elif hi:
            ins.append(f"v_xor_b32_e64 v{acc}, v{acc}, v{reg_h(hi)}")
        else:  # a nonzero c has an invertible matrix: no zero rows
            raise AssertionError("zero row for nonzero coefficient")
    ins.append(f"s_setpc_b64 s[{ret}:{ret + 1}]")
    ins.append("s_nop 0")
    return ins


def handler_table() -> list:
    """All handlers in address order: copy 0's c = 0..255, then copy 1's, ...
    Handler (copy k, coefficient c) lives at base + (256 k + c) * STRIDE."""
    return [i for k in range(NCOPY) for c in range(256) for i in handler(c, k)]


PLANE_REG = [reg_l(1), reg_l(2), reg_l(4), reg_l(8), reg_h(1), reg_h(2), reg_h(4), reg_h(8)]
STAGE = 24       # v[24:31]: next source's planes (staged layout: read one source ahead)
BANK = (64, 84)  # s[64:79] / s[84:99]: handler addresses of alternate sources
SM0 = 63         # m0 save
C = 8            # sources per LDS chunk (rs_tc.hip)
LDS_T = 2048     # LDS bytes per source: [2 halves][64 lanes] x 16 B
LDS_H = 1024


def chunk_v(nt: int) -> list:
    """chunk(nt) for nt <= 4 with the handler addresses taken from a VGPR
    instead of a scalar load (k_rs_tc_fused, which computes them itself):
    lane 16 t + i of %[av] holds dword i of source t's 8 addresses, moved into
    the source's SGPR bank by v_readlane_b32 where chunk() issues its
    s_load_dwordx16 (at least the 22 composites before the first use)."""
    assert 1 <= nt <= 4
    ins = chunk(nt)
    out = []
    for x in ins:
        if x.startswith("s_load_dwordx16"):
            bank = int(x.split("s[")[1].split(":")[0])
            off = x.rsplit(",", 1)[1].strip()
            t = 0 if off == "0" else int(off[3:-1])  # %[oN] -> N
            out += [f"v_readlane_b32 s{bank + i}, %[av], {16 * t + i}" for i in range(16)]
        else:
            out.append(x)
    return out


def chunk(nt: int) -> list:
    """One LDS chunk of nt sources in one asm statement (rs_tc.hip): every
    asynchronous load it issues is also waited for inside it.  Per source t:
    wait; move the staged planes into the table's single-bit entries; start
    source t+1's plane reads and handler-address load (other bank); build L/H;
    dispatch the 8 slots from this source's bank.
    Operands: %[la] = LDS byte address of the chunk + lane*16, %[pa] = address
    table of source 0 (this wave's 8 slots), %[o1].. = byte offsets of
    sources 1.. in that table."""
    def stage(t, dst=STAGE):
        return [f"ds_read_b128 v[{dst}:{dst + 3}], %[la] offset:{t * LDS_T}",
                f"ds_read_b128 v[{dst + 4}:{dst + 7}], %[la] offset:{t * LDS_T + LDS_H}"]

    def sload(t, bank):
        off = "0" if t == 0 else f"%[o{t}]"
        return [f"s_load_dwordx16 s[{bank}:{bank + 15}], %[pa], {off}"]

    late = LAYOUT == "late"
    ins = [f"s_mov_b32 s{SM0}, m0"] + sload(0, BANK[0]) + stage(0)
    for t in range(nt):
        cur, nxt = BANK[t & 1], BANK[(t + 1) & 1]
        ins.append("s_waitcnt lgkmcnt(0)")
        if not late:
            for a, r in enumerate(PLANE_REG):
                ins.append(f"v_mov_b32_e32 v{r}, v{STAGE + a}")
        if t + 1 < nt:
            ins += sload(t + 1, nxt) + ([] if late else stage(t + 1))
        ins += tables()
        # index mode on once per source; slots switch the index only
        mode = False
        for s0, ks, ix in GROUPS:
            if ix and not mode:
                ins.append(f"s_set_gpr_idx_on {ix}, gpr_idx(SRC0,DST)")
                mode = True
            elif ix:
                ins.append(f"s_set_gpr_idx_idx {ix}")
            for i in range(1, len(ks)):  # continuations of the chain
                ra, sl = RA_LIST[ks[i - 1]], s0 + i
                ins.append(f"s_mov_b64 s[{ra}:{ra + 1}], s[{cur + 2 * sl}:{cur + 2 * sl + 1}]")
            ins.append(f"s_swappc_b64 s[{RET}:{RET + 1}], s[{cur + 2 * s0}:{cur + 2 * s0 + 1}]")
        if mode:
            ins.append("s_set_gpr_idx_off")
        if late and t + 1 < nt:  # the planes are free once the dispatch is done
            ins += stage(t + 1)
    ins += [f"s_mov_b32 m0, s{SM0}", "s_nop 0"]
    return ins


def tables() -> list:
    """The 22 composite entries of the four-Russians tables."""
    ins = []
    for reg in (reg_l, reg_h):
        for n in range(1, 16):
            low = n & -n
            if n != low:
                ins.append(f"v_xor_b32_e32 v{reg(n)}, v{reg(n ^ low)}, v{reg(low)}")
    return ins


def main() -> None:
    out = sys.argv[1]
    lines = [
        "// generated by gen_tc_handlers.py -- do not edit",
        f"#define RSGPU_TC_STRIDE {STRIDE}",
        f"#define RSGPU_TC_ACC {ACC}",
        f"#define RSGPU_TC_LAYOUT_{LAYOUT.upper()} 1",
        f"#define RSGPU_TC_NHANDLERS {NHANDLERS}",
        "#define RSGPU_TC_SLOT_COPY {" + ", ".join(map(str, SLOT_COPY)) + "}",
        f"#define RSGPU_TC_RET {RET}",
        "#define RSGPU_TC_HANDLERS \\",
    ]
    for i in handler_table():
        lines.append(f'    "{i}\\n" \\')
    lines.append("")
    for nt in range(1, C + 1):
        lines.append(f"#define RSGPU_TC_CHUNK{nt} \\")
        for i in chunk(nt):
            lines.append(f'    "{i}\\n" \\')
        lines.append("")
    for nt in range(1, 5):
        lines.append(f"#define RSGPU_TC_CHUNKV{nt} \\")
        for i in chunk_v(nt):
            lines.append(f'    "{i}\\n" \\')
        lines.append("")
    lines.append(f"#define RSGPU_TC_C {C}")
    # the accumulators live only in asm-owned v[ACC:ACC+63] (the kernel caps
    # the compiler at v0..v{ACC-1}): zeroed, consumed and read out by asm
    lines.append("#define RSGPU_TC_ZERO \\")
    for i in range(0, 64, 2):  # v_mov_b64: two accumulator planes per instruction
        lines.append(f'    "v_mov_b64 v[{ACC + i}:{ACC + i + 1}], 0\\n" \\')
    lines.append("")
    for slot in range(8):
        body = "".join(f"v_mov_b32 %{q}, v{ACC + 8 * slot + q}\\n" for q in range(8))
        lines.append(f'#define RSGPU_TC_READ_SLOT{slot} "{body}"')
    for slot in range(8):  # the same with v_mov_b64 into 4 register pairs
        body = "".join(f"v_mov_b64 %{q}, v[{ACC + 8 * slot + 2 * q}:{ACC + 8 * slot + 2 * q + 1}]\\n"
                       for q in range(4))
        lines.append(f'#define RSGPU_TC_READ_SLOT64_{slot} "{body}"')
    for slot in range(8):
        body = "".join(f"v_mov_b32 v{ACC + 8 * slot + q}, %{q}\\n" for q in range(8))
        lines.append(f'#define RSGPU_TC_WRITE_SLOT{slot} "{body}"')
    for slot in range(8):
        a0 = ACC + 8 * slot
        lines.append(f'#define RSGPU_TC_LOAD_SLOT{slot} "global_load_dwordx4 v[{a0}:{a0 + 3}], %0, off\\n'
                     f'global_load_dwordx4 v[{a0 + 4}:{a0 + 7}], %0, off offset:16\\n"')
    lines.append("#define RSGPU_TC_ACC_CLOBBERS " + ", ".join(f'"v{ACC + i}"' for i in range(64)))
    # k_rs_jitw<R> (rs_jit.h Wide): R rows per wave, 8 R accumulators from v40
    A16 = 40
    for R in (16, 12, 10):
        lines.append(f"#define RSGPU_J{R}_ZERO \\")
        for i in range(0, 8 * R, 2):
            lines.append(f'    "v_mov_b64 v[{A16 + i}:{A16 + i + 1}], 0\\n" \\')
        lines.append("")
        lines.append(f"#define RSGPU_J{R}_ACC_CLOBBERS " + ", ".join(f'"v{A16 + i}"' for i in range(8 * R)))
    for slot in range(16):
        body = "".join(f"v_mov_b64 %{q}, v[{A16 + 8 * slot + 2 * q}:{A16 + 8 * slot + 2 * q + 1}]\\n"
                       for q in range(4))
        lines.append(f'#define RSGPU_JW_READ_SLOT64_{slot} "{body}"')
    lines.append("#define RSGPU_JW_CALL_CLOBBERS " + ", ".join(f'"v{r}"' for r in range(10, 40)))
    vclob = sorted(set(range(STAGE, STAGE + 8)) | set(TABLE_REGS))
    sclob = list(range(BANK[0], BANK[0] + 16)) + [SM0, RET, RET + 1] + list(range(BANK[1], BANK[1] + 16))
    for ra in RA_LIST:
        sclob += [ra, ra + 1]
    lines.append("#define RSGPU_TC_CLOBBERS " + ", ".join(
        [f'"v{r}"' for r in vclob] + [f'"s{r}"' for r in sclob] + ['"scc"']))
    lines.append("")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
