// jit_prog.cpp -- host-built generated code for a shared coefficient matrix
// (jit_prog.h).  Instruction encodings and the register contract: rs_jit.h.
#include "jit_prog.h"

#include <string.h>

#include <algorithm>

#include "rs_jit.h"
#include "rs_kernels.h"

namespace rsgpu {
namespace jit {

namespace {

// value id -> VGPR for a source in plane bank `bank`
inline int value_reg(int v, int bank) { return v < 8 ? plane_reg(bank, v) : 32 + (v - 8); }

// The full four-Russians tables (L[n] over planes 0-3, H[n] over 4-7, the 22
// composites of rs_jit.h's fixed layout) as a program: always a cover.
void full_tables(const uint8_t (&masks)[8 * kMaxSlots], int nm, SrcProg& p)
{
    uint8_t id[256];
    memset(id, kNone, sizeof id);
    for (int a = 0; a < 8; ++a)
        id[1 << a] = (uint8_t)a;
    p.nops = 0;
    for (int hi = 0; hi < 2; ++hi)
        for (int n = 1; n < 16; ++n) {
            const int low = n & -n;
            if (n == low)
                continue;
            const int sh = 4 * hi;
            p.ops[p.nops][0] = id[(n ^ low) << sh];
            p.ops[p.nops][1] = id[low << sh];
            p.ops[p.nops][2] = kNone;
            id[n << sh] = (uint8_t)(8 + p.nops);
            ++p.nops;
        }
    for (int i = 0; i < nm; ++i) {
        const int lo = masks[i] & 15, hi = masks[i] & 0xF0;
        p.outs[i][0] = lo ? id[lo] : (hi ? id[hi] : kNone);
        p.outs[i][1] = (lo && hi) ? id[hi] : kNone;
    }
}

}  // namespace

void plan_source(const uint8_t* coef, int nslot, SrcProg& p, int max_ops)
{
    uint8_t masks[8 * kMaxSlots];
    const int nm = 8 * nslot;
    for (int s = 0; s < nslot; ++s)
        for (int b = 0; b < 8; ++b)
            masks[8 * s + b] = mat_row(coef[s], b);
    // greedy cover (gen_enc_progs.py program()): values available so far,
    // have[m] = value id of mask m
    uint8_t have[256];
    memset(have, kNone, sizeof have);
    uint8_t vals[8 + kMaxComposites];
    int nv = 0;
    for (int a = 0; a < 8; ++a) {
        vals[nv] = (uint8_t)(1 << a);
        have[1 << a] = (uint8_t)nv++;
    }
    auto in = [&](int m) { return m == 0 || have[m] != kNone; };
    auto covered = [&](int m) {
        if (m == 0 || have[m] != kNone)
            return true;
        for (int i = 0; i < nv; ++i)
            if (have[m ^ vals[i]] != kNone)
                return true;
        return false;
    };
    bool need[256] = {};
    for (int i = 0; i < nm; ++i)
        if (!covered(masks[i]))
            need[masks[i]] = true;
    p.nops = 0;
    bool over = false;
    for (;;) {
        int nneed = 0;
        uint8_t nl[256];
        for (int m = 1; m < 256; ++m)
            if (need[m])
                nl[nneed++] = (uint8_t)m;
        if (!nneed)
            break;
        if (p.nops == max_ops || p.nops == kMaxComposites) {
            over = true;
            break;
        }
        bool cand[256] = {};
        for (int i = 0; i < nneed; ++i) {
            cand[nl[i]] = true;  // x ^ 0
            for (int j = 0; j < nv; ++j)
                cand[nl[i] ^ vals[j]] = true;
        }
        int best = -1, best_n = -1;
        uint8_t best_src[3] = {kNone, kNone, kNone};
        for (int c = 1; c < 256; ++c) {
            if (!cand[c] || have[c] != kNone)
                continue;
            uint8_t src[3] = {kNone, kNone, kNone};
            bool ok = false;
            for (int j = 0; j < nv && !ok; ++j) {  // one 2-input XOR of available values
                const int r = c ^ vals[j];
                if (r && have[r] != kNone) {
                    src[0] = (uint8_t)j;
                    src[1] = have[r];
                    ok = true;
                }
            }
            for (int j = 0; j < nv && !ok; ++j)  // or one 3-input XOR
                for (int l = j + 1; l < nv && !ok; ++l) {
                    const int r = c ^ vals[j] ^ vals[l];
                    if (r && r != vals[j] && r != vals[l] && have[r] != kNone) {
                        src[0] = (uint8_t)j;
                        src[1] = (uint8_t)l;
                        src[2] = have[r];
                        ok = true;
                    }
                }
            if (!ok)
                continue;
            int n = 0;
            for (int i = 0; i < nneed; ++i)
                n += nl[i] == c || in(nl[i] ^ c);
            if (n > best_n) {
                best = c;
                best_n = n;
                memcpy(best_src, src, 3);
            }
        }
        if (best < 0) {  // nothing buildable helps: fall back to the full tables
            over = true;
            break;
        }
        memcpy(p.ops[p.nops], best_src, 3);
        ++p.nops;
        vals[nv] = (uint8_t)best;
        have[best] = (uint8_t)nv++;
        for (int i = 0; i < nneed; ++i)
            if (covered(nl[i]))
                need[nl[i]] = false;
    }
    if (over) {
        full_tables(masks, nm, p);
        return;
    }
    for (int i = 0; i < nm; ++i) {
        const int m = masks[i];
        p.outs[i][0] = p.outs[i][1] = kNone;
        if (m == 0)
            continue;
        if (have[m] != kNone) {
            p.outs[i][0] = have[m];
            continue;
        }
        for (int j = 0; j < nv; ++j)
            if (have[m ^ vals[j]] != kNone) {
                p.outs[i][0] = (uint8_t)j;
                p.outs[i][1] = have[m ^ vals[j]];
                break;
            }
    }
}

int host_chunk_stride()
{
    const int per_src = 16 + 4 + 8 * kMaxComposites + 64 * 8;
    return (PRO_BYTES + 8 * per_src + EPI_BYTES + 63) / 64 * 64;
}

size_t emit_chunk(uint8_t* dst, int nt, int nslot, const SrcProg* progs)
{
    size_t o = 0;
    auto put32 = [&](uint32_t w) {
        memcpy(dst + o, &w, 4);
        o += 4;
    };
    auto put64 = [&](uint64_t w) {
        memcpy(dst + o, &w, 8);
        o += 8;
    };
    put64(enc_ds_read_b128(plane_reg(0, 0), 20, 0));
    put64(enc_ds_read_b128(plane_reg(0, 4), 20, LDS_HALF));
    for (int t = 0; t < nt; ++t) {
        const int bank = t & 1, nb = bank ^ 1;
        if (t + 1 < nt) {  // the next source's planes into the other bank
            put64(enc_ds_read_b128(plane_reg(nb, 0), 20, (t + 1) * LDS_SRC));
            put64(enc_ds_read_b128(plane_reg(nb, 4), 20, (t + 1) * LDS_SRC + LDS_HALF));
            put32(enc_waitcnt_lgkm(2));  // this source's two loads done
        } else {
            put32(enc_waitcnt_lgkm(0));
        }
        const SrcProg& p = progs[t];
        for (int i = 0; i < p.nops; ++i) {
            const int d = 32 + i, a = value_reg(p.ops[i][0], bank), b = value_reg(p.ops[i][1], bank);
            if (p.ops[i][2] == kNone)
                put32(enc_xor_e32(d, a, b));
            else
                put64(enc_bitop3_96(d, a, b, value_reg(p.ops[i][2], bank)));
        }
        for (int s = 0; s < nslot; ++s)
            for (int b = 0; b < 8; ++b) {
                const uint8_t* q = p.outs[8 * s + b];
                const int acc = ACC + 8 * s + b;
                if (q[0] == kNone)
                    continue;  // zero mask: nothing to add
                if (q[1] == kNone)
                    put64(enc_xor_e64(acc, acc, value_reg(q[0], bank)));
                else
                    put64(enc_bitop3_96(acc, acc, value_reg(q[0], bank), value_reg(q[1], bank)));
            }
    }
    put64((uint64_t)S_NOP0 << 32 | S_SETPC_82);
    return o;
}

std::vector<uint8_t> build_matrix_code(const uint8_t* c, int k, int e, int* chunk_stride, int max_ops)
{
    const int stride = host_chunk_stride(), nch = (k + 7) / 8, passes = (e + 31) / 32;
    *chunk_stride = stride;
    std::vector<uint8_t> code((size_t)passes * 4 * nch * stride);
    // unused bytes: returns (a call that lands there comes straight back)
    for (size_t i = 0; i + 8 <= code.size(); i += 8) {
        const uint64_t ret = (uint64_t)S_NOP0 << 32 | S_SETPC_82;
        memcpy(&code[i], &ret, 8);
    }
    SrcProg progs[8];
    for (int p = 0; p < passes; ++p) {
        const int rows = std::min(32, e - 32 * p), nw = (rows + 7) / 8;
        for (int w = 0; w < nw; ++w) {
            const int nslot = std::min(8, rows - 8 * w);
            for (int ch = 0; ch < nch; ++ch) {
                const int nt = std::min(8, k - 8 * ch);
                for (int t = 0; t < nt; ++t) {
                    uint8_t cf[8];
                    for (int s = 0; s < nslot; ++s)
                        cf[s] = c[(size_t)(32 * p + 8 * w + s) * k + 8 * ch + t];
                    plan_source(cf, nslot, progs[t], max_ops);
                }
                emit_chunk(&code[(((size_t)p * 4 + w) * nch + ch) * stride], nt, nslot, progs);
            }
        }
    }
    return code;
}

namespace {

// value id -> VGPR in the two-wave layout (rs_jit.h Wide)
inline int wide_reg(int v) { return v < 8 ? 10 + v : 18 + (v - 8); }

// One chunk of the two-wave layout at dst (nullptr: size only).
size_t emit_chunk_wide(uint8_t* dst, int nt, int nslot, const SrcProg* progs)
{
    size_t o = 0;
    auto put32 = [&](uint32_t w) {
        if (dst)
            memcpy(dst + o, &w, 4);
        o += 4;
    };
    auto put64 = [&](uint64_t w) {
        if (dst)
            memcpy(dst + o, &w, 8);
        o += 8;
    };
    for (int t = 0; t < nt; ++t) {
        put64(enc_ds_read_b128(10, 9, t * LDS_SRC));
        put64(enc_ds_read_b128(14, 9, t * LDS_SRC + LDS_HALF));
        put32(enc_waitcnt_lgkm(0));
        const SrcProg& p = progs[t];
        for (int i = 0; i < p.nops; ++i) {
            const int d = 18 + i, a = wide_reg(p.ops[i][0]), b = wide_reg(p.ops[i][1]);
            if (p.ops[i][2] == kNone)
                put32(enc_xor_e32(d, a, b));
            else
                put64(enc_bitop3_96(d, a, b, wide_reg(p.ops[i][2])));
        }
        for (int s = 0; s < nslot; ++s)
            for (int b = 0; b < 8; ++b) {
                const uint8_t* q = p.outs[8 * s + b];
                const int acc = 40 + 8 * s + b;
                if (q[0] == kNone)
                    continue;  // zero mask: nothing to add
                if (q[1] == kNone)
                    put64(enc_xor_e64(acc, acc, wide_reg(q[0])));
                else
                    put64(enc_bitop3_96(acc, acc, wide_reg(q[0]), wide_reg(q[1])));
            }
    }
    put64((uint64_t)S_NOP0 << 32 | S_SETPC_82);
    return o;
}

}  // namespace

std::vector<uint8_t> build_matrix_code_wide(const uint8_t* c, int k, int e, int R, int CS, int* chunk_stride,
                                            int max_ops)
{
    const int nch = (k + CS - 1) / CS;
    // programs of every (wave, source), then the chunk sizes
    const int nv = wide_waves(e);
    auto row0 = [&](int w) { return wide_row0(e, w); };
    if ((e + nv - 1) / nv > R || R > kMaxSlots)  // a wave's rows exceed its accumulators
        return {};
    std::vector<SrcProg> progs((size_t)nv * k);
    for (int w = 0; w < nv; ++w) {
        const int nslot = row0(w + 1) - row0(w);
        for (int q = 0; q < k && nslot > 0; ++q) {
            uint8_t cf[kMaxSlots];
            for (int s = 0; s < nslot; ++s)
                cf[s] = c[(size_t)(row0(w) + s) * k + q];
            plan_source(cf, nslot, progs[(size_t)w * k + q], max_ops);
        }
    }
    size_t most = 0;
    for (int w = 0; w < nv; ++w) {
        const int nslot = row0(w + 1) - row0(w);
        for (int ch = 0; ch < nch && nslot > 0; ++ch)
            most = std::max(most, emit_chunk_wide(nullptr, std::min(CS, k - CS * ch), nslot,
                                                  &progs[(size_t)w * k + CS * ch]));
    }
    const int stride = (int)((most + 63) / 64 * 64);
    *chunk_stride = stride;
    std::vector<uint8_t> code((size_t)nv * nch * stride);
    for (size_t i = 0; i + 8 <= code.size(); i += 8) {
        const uint64_t ret = (uint64_t)S_NOP0 << 32 | S_SETPC_82;
        memcpy(&code[i], &ret, 8);
    }
    for (int w = 0; w < nv; ++w) {
        const int nslot = row0(w + 1) - row0(w);
        for (int ch = 0; ch < nch && nslot > 0; ++ch)
            emit_chunk_wide(&code[((size_t)w * nch + ch) * stride], std::min(CS, k - CS * ch), nslot,
                            &progs[(size_t)w * k + CS * ch]);
    }
    return code;
}

std::vector<uint8_t> build_matrix_code_wide_passes(const uint8_t* c, int k, int e,
                                                   std::vector<std::pair<size_t, int>>* passes, int max_ops)
{
    std::vector<uint8_t> code;
    passes->clear();
    for (int p = 0; p < wide_passes(e); ++p) {
        const int r0 = wide_pass_row0(e, p), pr = wide_pass_rows(e, p);
        int stride = 0;
        const std::vector<uint8_t> cp =
            build_matrix_code_wide(c + (size_t)r0 * k, k, pr, jitw_rows(pr), jitw_cs(pr), &stride, max_ops);
        if (cp.empty())
            return {};
        passes->push_back({code.size(), stride});
        code.insert(code.end(), cp.begin(), cp.end());
    }
    return code;
}

}  // namespace jit
}  // namespace rsgpu
