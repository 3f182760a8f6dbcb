// rs_bitsliced.hip -- bit-sliced RS(K, E) parity kernel with
// compile-time coefficients (the gf_gen_rs_matrix code, isa/ec_base.c:62-79).
//
// Why bit-slicing: on gfx950 a wave64 v_bitop3/v_xor/v_and issues in ~2
// cycles per SIMD but v_perm/v_pk_*/v_bfi in ~4 (profiles/r1_ubench_valu.log),
// and the GF(2^8) product by a constant is GF(2)-linear.  With each lane
// holding 32 consecutive bytes of a row as 8 bit-planes (plane a = bit a of
// the 32 bytes), multiplying by a constant c and accumulating is, per output
// plane, one 3-input XOR of two "four Russians" entries
//     out_b ^= L[m_b & 15] ^ H[m_b >> 4],
// L[n] = XOR of planes 0..3 selected by n, H[n] = same for planes 4..7, m_b =
// row b of c's 8x8 bit matrix.  That is 8 full-rate ops per (coefficient,
// 32 bytes) versus 24 quarter-rate v_perm for the same bytes.  With the
// coefficients known at compile time, only the composites a block of rows
// actually uses are built (gen_enc_progs.py: a greedy cover, 10.9 instead of
// 22 per source on average; the encode measured 2.7 % faster).
//
// Code size: the parity matrix has entries 2^(r*j).  Sources are processed in
// chunks of C with Horner's rule over chunks,
//     p_r = sum_c 2^(C r c) * E_c(r),   E_c(r) = sum_t 2^(r t) d_{cC+t},
// so one chunk's straight-line code (coefficients 2^(r t), t < C) serves
// every chunk; between chunks each accumulator is multiplied by the constant
// 2^(C r) (~16 XORs).  The chunk loop is a runtime loop.  A chunk's source 0
// has the coefficient 1 on every row: its single-plane terms ride along in
// the 3-input XOR of a later source whose term is a single value too
// (T0Pair, gen_enc_progs.py), 3 % fewer instructions at (64, 32).
//
// Work split: a workgroup of NW waves shares 64 x 32 = 2048 byte positions;
// wave w owns outputs [w*OPW, (w+1)*OPW) (8 planes x OPW accumulators in
// VGPRs, <= 128 VGPRs for 4 waves/SIMD).  The NW waves divide each chunk's
// sources for loading + transposing into LDS, then all read every source's
// planes from LDS.  Bit transposes are SWAR 8x8 bit-matrix transposes across
// the lane's 8 dwords (12 block swaps), and the same routine converts the
// accumulators back to bytes.
//
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "bitslice.h"
#include "diag_clock.h"
#include "gf256.h"
#include "kernel_hooks.h"
#include "rs_kernels.h"

namespace rsgpu {
namespace bs {

RSGPU_DIAG_TABLE

template <int K, int E, int C>
struct PlanHolder {  // the code (K, E) and its Horner chunk C
    static constexpr int k = K, e = E, c = C;
};

// Per-source XOR programs (gen_enc_progs.py -> build/enc_progs.inc): for
// rows R0..R0+NR-1 at chunk position T, the composite XORs of the source
// planes that the block's masks need (values 8..), and for every output
// plane the one or two values it adds.
template <int K, int E, int C, int R0, int NR, int T>
struct EncProg;
template <int K, int E, int C, int R>
struct TwProg;
template <int K, int E, int C, int R0, int NR>
struct T0Pair;
#include "enc_progs.inc"

template <class PR, int I, int NV>
__device__ __forceinline__ void prog_op(uint32_t (&V)[NV]);

// row R's accumulator times 2^(C R): the generated XOR program over its 8
// planes (TwProg, gen_enc_progs.py)
template <class P, int R, int... Bs>
__device__ __forceinline__ void twiddle_row(uint32_t (&acc)[8], std::integer_sequence<int, Bs...>)
{
    using PR = TwProg<P::k, P::e, P::c, R>;
    uint32_t V[8 + PR::NOPS];
#pragma unroll
    for (int a = 0; a < 8; ++a)
        V[a] = acc[a];
    [&]<int... Is>(std::integer_sequence<int, Is...>) {
        (prog_op<PR, Is>(V), ...);
    }(std::make_integer_sequence<int, PR::NOPS>{});
    ((acc[Bs] = V[PR::outs[Bs]]), ...);
}

template <class P, int R0, int NR, int... Rs>
__device__ __forceinline__ void twiddle_rows(uint32_t (&acc)[NR][8], std::integer_sequence<int, Rs...>)
{
    (twiddle_row<P, R0 + Rs>(acc[Rs], std::make_integer_sequence<int, 8>{}), ...);
}

template <class PR, int I, int NV>
__device__ __forceinline__ void prog_op(uint32_t (&V)[NV])
{
    constexpr int a = PR::ops[I][0], b = PR::ops[I][1], c = PR::ops[I][2];
    if constexpr (c == 255)
        V[8 + I] = V[a] ^ V[b];
    else
        V[8 + I] = x3(V[a], V[b], V[c]);
}

// Output O of source T: its one or two values; source 0's single plane
// moves to the partner source of T0Pair (one 3-input XOR for both terms)
template <class PR, class PP, bool PAIR, int T, int O, int NV>
__device__ __forceinline__ void prog_out(uint32_t& acc, const uint32_t (&V)[NV], const uint32_t (&p0)[8])
{
    constexpr int x = PR::outs[O][0], y = PR::outs[O][1];
    constexpr int partner = PAIR ? PP::partner[O] : 0;  // 0: source 0 adds its own plane
    if constexpr (T == 0 && partner != 0) {
        // added by source `partner`
    } else if constexpr (T != 0 && partner == T) {
        static_assert(x != 255 && y == 255, "T0 partner output must be a single value");
        acc = x3(acc, V[x], p0[O % 8]);
    } else if constexpr (x != 255 && y != 255) {
        acc = x3(acc, V[x], V[y]);
    } else if constexpr (x != 255) {
        acc ^= V[x];
    }
}

// consume source T of the chunk from planes p (all lanes), for this wave's
// rows: the generated program's composites, then one XOR per output plane
// (p0: the chunk's source 0 planes, for the outputs paired with it)
template <class P, int R0, int NR, int T, bool PAIR = true>
__device__ __forceinline__ void consume(uint32_t (&acc)[NR][8], const uint32_t (&p)[8], const uint32_t (&p0)[8])
{
    using PR = EncProg<P::k, P::e, P::c, R0, NR, T>;
    using PP = T0Pair<P::k, P::e, P::c, R0, NR>;
    constexpr int NV = 8 + PR::NOPS;
    uint32_t V[NV];
#pragma unroll
    for (int a = 0; a < 8; ++a)
        V[a] = p[a];
    [&]<int... Is>(std::integer_sequence<int, Is...>) {
        (prog_op<PR, Is>(V), ...);
    }(std::make_integer_sequence<int, PR::NOPS>{});
    [&]<int... Os>(std::integer_sequence<int, Os...>) {
        (prog_out<PR, PP, PAIR, T, Os>(acc[Os / 8][Os % 8], V, p0), ...);
    }(std::make_integer_sequence<int, NR * 8>{});
}

struct Args {
    const uint8_t* src;   // [B][K] rows
    uint8_t* out;         // [B][E] rows
    long long pitch, len;
    long long blocks;     // B
    int flat;             // tiles over the blocks' rows laid end to end (short rows)
    int prio;             // A/B: wave priority level from the transposes to the part barrier
};

// Where lane `lane` of column tile `tile` works: the tile's first block b0,
// the lane's block b0 + db and byte offset o in its rows, and whether it has
// bytes at all.  Per block, tiles cover [0, len) in 2 KB steps, the last one
// partial (C4: 32000 = 15 x 2048 + 1280, 2.4 % of the tiles' lanes idle).
// flat: tiles cover the B blocks' rows as one run of B x len bytes per row
// index (len % 32 == 0, so a lane's 32 bytes never straddle two blocks) and
// a tile's lanes may belong to consecutive blocks: one idle tail per launch.
struct TilePos {
    long long b0, o;
    int db;
    bool inb;
};
__device__ __forceinline__ TilePos tile_pos(const Args& a, int lane)
{
    TilePos p;
    if (!a.flat) {
        p.b0 = blockIdx.y;
        p.o = (long long)blockIdx.x * 2048 + lane * 32;
        p.db = 0;
        p.inb = p.o + 32 <= a.len;
        return p;
    }
    const long long t0 = (long long)blockIdx.x * 2048;
    p.b0 = t0 / a.len;                                // wave-uniform
    const int x = (int)(t0 - p.b0 * a.len) + lane * 32;  // < len + 2048 < 2^24
    int db = (int)((float)x * (1.0f / (float)a.len));
    const int L = (int)a.len;
    if (x - db * L >= L)
        ++db;
    if (x - db * L < 0)
        --db;
    p.db = db;
    p.o = x - (long long)db * L;
    p.inb = p.b0 + db < a.blocks;
    return p;
}

// LDS part: S sources of [2 halves][64 lanes] x 16 B; two parts double-buffer
// the source stream (2 x 16 KiB).  A plan chunk of C sources is ceil(C/S)
// consecutive parts.
constexpr int S = 8;

// Sources T = PART*S + t (t < S, T < C) of the current chunk from the LDS part.
template <class P, int K, int C, int R0, int NR, int PART>
__device__ __forceinline__ void consume_part(uint32_t (&acc)[NR][8], uint32_t (&p0)[8], const uint4* buf,
                                             int lane, int j0)
{
    [[maybe_unused]] uint32_t zp[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // kernel_hooks.h kZeroValuPlanes only
    [&]<int... Ts>(std::integer_sequence<int, Ts...>) {
        (
            [&] {
                constexpr int T = PART * S + Ts;
                if constexpr (T < C) {
                    if (j0 + Ts < K) {
                        const uint4 u = buf[(Ts * 2 + 0) * 64 + lane];
                        const uint4 v = buf[(Ts * 2 + 1) * 64 + lane];
                        uint32_t pl[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
                        if constexpr (Hooks::kZeroValuPlanes) {
                            // the reads kept, the VALU fed zeros that are new values to
                            // the compiler per source (no instruction, no CSE)
                            asm volatile("" ::"v"(u.x), "v"(u.y), "v"(u.z), "v"(u.w), "v"(v.x), "v"(v.y), "v"(v.z),
                                         "v"(v.w));
                            asm volatile("" : "+v"(zp[0]), "+v"(zp[1]), "+v"(zp[2]), "+v"(zp[3]), "+v"(zp[4]),
                                         "+v"(zp[5]), "+v"(zp[6]), "+v"(zp[7]));
#pragma unroll
                            for (int a = 0; a < 8; ++a)
                                pl[a] = zp[a];
                        }
                        if constexpr (T == 0) {
#pragma unroll
                            for (int a = 0; a < 8; ++a)
                                p0[a] = pl[a];
                        }
                        consume<P, R0, NR, T>(acc, pl, p0);
                    }
                    // keep the next source's LDS reads from being hoisted
                    // here (they would pin 8 more VGPRs per source)
                    __builtin_amdgcn_sched_barrier(0);
                }
            }(),
            ...);
    }(std::make_integer_sequence<int, S>{});
}

// One wave group: rows [R0, R0+NR).  The workgroup streams the sources
// chunk by chunk (Horner order, last chunk first) through the LDS parts:
// while part n is transposed in place and consumed, part n+1 is already in
// flight by LDS-DMA (global_load_lds_dwordx4, counted vmcnt, raw barriers).
template <int K, int E, int C, int NW, int G, bool PRIO>
__device__ __forceinline__ void run_group(const Args& a, uint4 (*lds)[S * 2 * 64])
{
    using P = PlanHolder<K, E, C>;
    constexpr int OPW = (E + NW - 1) / NW;
    constexpr int R0 = G * OPW;
    constexpr int NR = (E - R0) < OPW ? (E - R0) : OPW;
    constexpr int NCH = (K + C - 1) / C;
    constexpr int NP = (C + S - 1) / S;  // parts per chunk
    static_assert(NR > 0, "empty wave group");

    const int lane = threadIdx.x & 63;
    const TilePos tp = tile_pos(a, lane);
    const bool inb = tp.inb;
    // source offset from the tile's first block; out-of-range lanes re-read
    // the row head
    // (kernel_hooks.h: the diagnostic HBM-quiet variant moves both into a
    // two-block window)
    const long long wo = Hooks::data_offset(tp.o, blockIdx.x, lane);
    const long long wb = Hooks::data_block(tp.b0);
    const long long loff = inb ? tp.db * (long long)K * a.pitch + wo : 0;
    const uint8_t* sb = a.src + (size_t)wb * K * a.pitch;
    auto live = [&](int j) { return j < K; };
    const uint32_t m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)&lds[0][0];

    // step n -> (chunk, part): chunks in Horner order NCH-1 .. 0
    constexpr int NSTEP = NCH * NP;
    auto first_src = [&](int n) { return (NCH - 1 - n / NP) * C + (n % NP) * S; };
    auto part_len = [&](int n) {
        const int p = n % NP;
        return min(S, C - p * S);
    };
    // this wave's share of step n: t = G, G + NW, ...
    auto issue = [&](int n) {
        const int j0 = first_src(n), nt = part_len(n);
        const uint32_t base = lds0 + (uint32_t)((n & 1) * S * 2 * 64 * 16);
        for (int t = G; t < nt; t += NW)
            if (live(j0 + t))
                bs::glds32(sb + (size_t)(j0 + t) * a.pitch, (uint32_t)loff,
                           base + (uint32_t)(t * 2 * 64 * 16));
    };
    auto issued = [&](int n) {
        const int j0 = first_src(n), nt = part_len(n);
        int c = 0;
        for (int t = G; t < nt; t += NW)
            c += live(j0 + t) ? 2 : 0;
        return c;
    };

    uint32_t acc[NR][8];
    uint32_t p0[8] = {};  // planes of the current chunk's source 0 (T0Pair)
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q)
            acc[r][q] = 0;

    issue(0);
    for (int n = 0; n < NSTEP; ++n) {
        uint4* buf = lds[n & 1];
        const int j0 = first_src(n), nt = part_len(n);
        if (n + 1 < NSTEP) {
            issue(n + 1);
            bs::wait_vm(issued(n + 1));
        } else {
            bs::wait_vm(0);
        }
        // the transposes up to the part barrier over the other workgroups'
        // multiply-accumulates (round 6, profiles/r06_prio/: encode -1.2 to -2.3 %)
        if constexpr (PRIO)
            asm volatile("s_setprio 2" ::: "memory");
        for (int t = G; t < nt; t += NW)
            if (live(j0 + t)) {
                uint4 u = buf[(t * 2 + 0) * 64 + lane];
                uint4 v = buf[(t * 2 + 1) * 64 + lane];
                uint32_t W[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
                if constexpr (!Hooks::kTransposes)
                    continue;
                tr8(W, m4, m2, m1);
                hook_planes<Hooks>(W);
                buf[(t * 2 + 0) * 64 + lane] = make_uint4(W[0], W[1], W[2], W[3]);
                buf[(t * 2 + 1) * 64 + lane] = make_uint4(W[4], W[5], W[6], W[7]);
            }
        bs::barrier_lds();
        if constexpr (PRIO)
            asm volatile("s_setprio 0" ::: "memory");
        const int part = n % NP;
        if (part == 0 && n != 0)
            twiddle_rows<P, R0, NR>(acc, std::make_integer_sequence<int, NR>{});
        // consume part `part` of the chunk: compile-time T = part*S + t
        [&]<int... Ps>(std::integer_sequence<int, Ps...>) {
            ((part == Ps ? consume_part<P, K, C, R0, NR, Ps>(acc, p0, buf, lane, j0)
                         : void()),
             ...);
        }(std::make_integer_sequence<int, NP>{});
        bs::barrier_lds();  // part buffer n & 1 is refilled by step n + 2
    }

    if (!inb)
        return;
    uint8_t* ob = a.out + (size_t)wb * E * a.pitch;
    const long long ooff = tp.db * (long long)E * a.pitch + wo;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        uint32_t W[8];
#pragma unroll
        for (int q = 0; q < 8; ++q)
            W[q] = acc[r][q];
        tr8(W, m4, m2, m1);
        store32(ob + (size_t)(R0 + r) * a.pitch, ooff, W);
    }
}

// waves per SIMD the register budget must allow: 4 while a wave owns <= 8 rows
// (64 accumulator VGPRs), 2 for 16 rows (128 accumulators; halves the
// per-wave four-Russians table builds, but measured slower at (64, 32):
// 24.2 vs 23.2 ms, two waves per SIMD do not hide the LDS-DMA pipeline)
template <int E, int NW>
constexpr int bs_waves_per_simd()
{
    return (E + NW - 1) / NW > 8 ? 2 : 16 / NW;
}

template <int K, int E, int C, int NW, bool PRIO = true>
__global__ __launch_bounds__(64 * NW, (bs_waves_per_simd<E, NW>())) void k_rs_bs(Args a)
{
    __shared__ uint4 lds[2][S * 2 * 64];
    RSGPU_DIAG_BEGIN()
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    [&]<int... Gs>(std::integer_sequence<int, Gs...>) {
        ((wave == Gs ? run_group<K, E, C, NW, Gs, PRIO>(a, lds) : void()), ...);
    }(std::make_integer_sequence<int, NW>{});
    RSGPU_DIAG_END();
}

// Small batches of a single-chunk code (C == K, E <= 8; C2: one block of
// (16, 4, 1e6), 489 tiles, where one wave per tile leaves most SIMDs idle
// and walks all K sources in series): SPL waves split a tile's sources,
// wave w taking T = w, w + SPL, ... with the compile-time programs of those
// T (no source 0 pairing: the partner may belong to another wave), straight
// from global memory into registers; the partial accumulators meet in LDS
// and wave w finishes rows w, w + SPL, ...
template <int K, int E, int SPL, int G>
__device__ __forceinline__ void split_group(const Args& a, uint32_t (&acc)[E][8], long long loff)
{
    using P = PlanHolder<K, E, K>;
    const uint8_t* sb = a.src + (size_t)blockIdx.y * K * a.pitch;
    constexpr int NT = (K - G + SPL - 1) / SPL;  // this wave's sources
    uint32_t W[NT][8];
#pragma unroll
    for (int i = 0; i < NT; ++i)  // every load in flight before the first use
        load32(sb + (size_t)(G + SPL * i) * a.pitch, loff, true, W[i]);
    const uint32_t m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);
    const uint32_t none[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    [&]<int... Is>(std::integer_sequence<int, Is...>) {
        (
            [&] {
                tr8(W[Is], m4, m2, m1);
                consume<P, 0, E, G + SPL * Is, false>(acc, W[Is], none);
            }(),
            ...);
    }(std::make_integer_sequence<int, NT>{});
}

template <int K, int E, int SPL>
__global__ __launch_bounds__(64 * SPL) void k_rs_bs_split(Args a)
{
    static_assert(E <= 8 && K >= SPL, "split encode: one row group, every wave a source");
    __shared__ uint32_t part[SPL][E * 8][64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long long off = (long long)blockIdx.x * 2048 + lane * 32;
    const bool inb = off + 32 <= a.len;
    const long long loff = inb ? off : 0;  // out-of-range lanes re-read the row head
    uint32_t acc[E][8];
#pragma unroll
    for (int r = 0; r < E; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q)
            acc[r][q] = 0;
    [&]<int... Gs>(std::integer_sequence<int, Gs...>) {
        ((wave == Gs ? split_group<K, E, SPL, Gs>(a, acc, loff) : void()), ...);
    }(std::make_integer_sequence<int, SPL>{});
#pragma unroll
    for (int r = 0; r < E; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q)
            part[wave][r * 8 + q][lane] = acc[r][q];
    __syncthreads();
    if (!inb)
        return;
    const uint32_t m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);
    uint8_t* ob = a.out + (size_t)blockIdx.y * E * a.pitch;
    for (int r = wave; r < E; r += SPL) {
        uint32_t W[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int w = 0; w < SPL; ++w)
#pragma unroll
            for (int q = 0; q < 8; ++q)
                W[q] ^= part[w][r * 8 + q][lane];
        tr8(W, m4, m2, m1);
        store32(ob + (size_t)r * a.pitch, off, W);
    }
}

template <int K, int E>
hipError_t launch_split(const uint8_t* src, uint8_t* out, long long pitch, long long len, long long blocks,
                        hipStream_t st)
{
    Args a{src, out, pitch, len, blocks, 0};
    dim3 grid((unsigned)((len + 2047) / 2048), (unsigned)blocks);
    hipLaunchKernelGGL((k_rs_bs_split<K, E, 4>), grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Small decode batches of a single-chunk compiled code (C2: one block of
// (16, 4, 1e6)): syndromes through the encode's compile-time programs, then
// the e x e solve with runtime coefficients, in ONE launch.
//
// isa.cpp:169-213 applies rows of inv(b); the erased originals E also solve
// d_E = V_E^-1 s with s = P ^ V_Ebar d_Ebar (the same unique
// bytes).  V_Ebar holds the code's own entries 2^(p j), so each surviving
// original goes through consume<> exactly as in the encode (a uniform branch
// skips an erased one) and the parity rows are XORed in: no closed form and
// no threaded code for the e x k part.  Row i of V_E^-1 is [z^p] Q_i(z) / w_i,
// Q_i = prod_{l != i} (z + a_l), a_l = 2^(j_l), w_i = Q_i(a_i), built
// lane-parallel while the sources fly (lane 8 i + m: [z^m] Q_i, as
// k_rs_tc_fused builds its parity coefficients).  A runtime coefficient c
// applies through its 8 x 8 bit matrix: plane b of c x is the XOR over a of
// plane a of x where bit b of c 2^a is set, one v_bitop3 (out ^ (s & mask),
// mask an SGPR of 0 or ~0) per (a, b).  Four waves per 2 KB tile split the
// sources as k_rs_bs_split; the partial syndromes meet in LDS, each wave
// XORing its partials into one zeroed copy (ds_xor_b32), so the output phase
// reads every syndrome once instead of once per wave: C2 698-701 vs 687-689
// GiB/s, same box x4 (profiles/r04_spl/ldsx_*).
alignas(16) __device__ const GfTables kGfBs = make_gf_tables();

// parity rows p = G, G + SPL, ... of wave G: they survive whatever the
// erasure list says, so their loads go out before the list arrives
template <int E, int SPL, int G>
__device__ __forceinline__ void syn_parity_loads(const SynArgs& a, long long loff, uint32_t (&Pw)[2][8])
{
    constexpr int NP = (E - G + SPL - 1) / SPL;
    static_assert(NP <= 2, "two parity rows per wave at most");
#pragma unroll
    for (int i = 0; i < NP; ++i)
        load32(a.par + ((size_t)blockIdx.y * E + G + SPL * i) * a.pitch, loff, true, Pw[i]);
}

template <class F, int K, int E, int SPL, int G>
__device__ __forceinline__ void syn_group(const SynArgs& a, unsigned long long emask, long long loff,
                                          uint32_t (&acc)[E][8], uint32_t (&Pw)[2][8], F&& between)
{
    using P = PlanHolder<K, E, K>;
    const int b = blockIdx.y;
    const uint8_t* sb = a.src + (size_t)b * K * a.pitch;
    constexpr int NT = (K - G + SPL - 1) / SPL;  // this wave's sources T = G, G + SPL, ...
    constexpr int NP = (E - G + SPL - 1) / SPL;  // its parity rows p = G, G + SPL, ...
    uint32_t W[NT][8];
    // every source load in flight at once; an erased original is never read
#pragma unroll
    for (int i = 0; i < NT; ++i)
        load32(sb + (size_t)(G + SPL * i) * a.pitch, loff, !((emask >> (G + SPL * i)) & 1), W[i]);
    between();  // the solve's coefficients, while the loads fly
    const uint32_t m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);
    const uint32_t none[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    [&]<int... Is>(std::integer_sequence<int, Is...>) {
        (
            [&] {
                constexpr int T = G + SPL * Is;
                if (!((emask >> T) & 1)) {
                    tr8(W[Is], m4, m2, m1);
                    consume<P, 0, E, T, false>(acc, W[Is], none);
                }
            }(),
            ...);
    }(std::make_integer_sequence<int, NT>{});
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        tr8(Pw[i], m4, m2, m1);
#pragma unroll
        for (int q = 0; q < 8; ++q)
            acc[G + SPL * i][q] ^= Pw[i][q];
    }
}

template <int K, int E, int SPL>
__global__ __launch_bounds__(64 * SPL) void k_rs_syn_split(SynArgs a)
{
    static_assert(E <= 8 && K <= 64 && K >= SPL, "one chunk, e <= 8");
    __shared__ uint32_t syn[E * 8][64];  // the syndromes: every wave's partials XORed in
    __shared__ uint32_t gtw[SPL][192];  // per wave: exp[512] | log[256]
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.y;
    const long long off = (long long)blockIdx.x * 2048 + lane * 32;
    const bool inb = off + 32 <= a.len;
    const long long loff = inb ? off : 0;  // out-of-range lanes re-read the row head
    uint32_t Pw[2][8];
    [&]<int... Gs>(std::integer_sequence<int, Gs...>) {
        ((wave == Gs ? syn_parity_loads<E, SPL, Gs>(a, loff, Pw) : void()), ...);
    }(std::make_integer_sequence<int, SPL>{});
    for (int i = threadIdx.x; i < E * 8 * 64; i += 64 * SPL)
        (&syn[0][0])[i] = 0;
    __syncthreads();
    // the GF tables and the block's erasure list in one round trip
    const uint32_t* tsrc = reinterpret_cast<const uint32_t*>(&kGfBs);
    const uint32_t t0 = tsrc[lane], t1 = tsrc[64 + lane], t2 = tsrc[128 + lane];
    // lane i: erased original j_i.  The block's list through the scalar
    // cache: the aligned words holding its E bytes (never past the word that
    // holds the last one); C2 678-680 vs 674-676 GiB/s with a vector load,
    // same box x4 (profiles/r04_slist/)
    int j;
    {
        typedef const uint32_t __attribute__((address_space(4)))* CW;
        const uint8_t* lp = a.err + (size_t)b * E;  // any alignment (a slice's list)
        const size_t off = (uintptr_t)lp & 3;
        const CW wp = (CW)(lp - off);
        constexpr int NW = (3 + E + 3) / 4;
        uint32_t w[NW];
#pragma unroll
        for (int i = 0; i < NW; ++i)
            w[i] = (off + E + 3) / 4 > (size_t)i ? wp[i] : 0u;
        const int p = (int)off + lane;  // this lane's byte
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i)
            v = (p >> 2) == i ? w[i] : v;
        j = lane < E ? (int)((v >> (8 * (p & 3))) & 0xFFu) : 255;
    }
    const int jp = __shfl_up(j, 1);
    if (__ballot(lane < E && (j >= K || (lane > 0 && j <= jp))) != 0) {  // strictly ascending, < k
        if (blockIdx.x == 0 && threadIdx.x == 0)
            a.status[b] = -2;
        return;  // uniform per workgroup
    }
    bool er = false;
#pragma unroll
    for (int i = 0; i < E; ++i)
        er |= __builtin_amdgcn_readlane(j, i) == lane;
    const unsigned long long emask = __ballot(lane < K && er);
    uint32_t* gw = gtw[wave];
    gw[lane] = t0;
    gw[64 + lane] = t1;
    gw[128 + lane] = t2;
    const uint8_t* gexp = reinterpret_cast<const uint8_t*>(gw);
    const uint8_t* glog = gexp + 512;
    int coef = 0;  // lane 8 i + m: (V_E^-1)[i][m]
    auto solve_rows = [&] {
        const int i = lane >> 3, m = lane & 7;
        int J[8], A[8];
#pragma unroll
        for (int l = 0; l < 8; ++l)
            J[l] = __builtin_amdgcn_readlane(j, l);
        const int al = lane < E ? gexp[j] : 0;
#pragma unroll
        for (int l = 0; l < 8; ++l)
            A[l] = __builtin_amdgcn_readlane(al, l);
        int ji = 0, ai = 0;
#pragma unroll
        for (int l = 0; l < 8; ++l) {
            ji = i == l ? J[l] : ji;
            ai = i == l ? A[l] : ai;
        }
        const int tv = gexp[(ji + m) % 255];  // lane 8 l + c: a_l 2^c = 2^(j_l + c)
        int qv = m == 0;                      // Q_i, one factor (z + a_l) at a time
#pragma unroll
        for (int l = 0; l < E; ++l) {
            int pr = 0;  // a_l q_m from the 2^c multiples of a_l where q_m has bit c
#pragma unroll
            for (int c = 0; c < 8; ++c)
                pr ^= __builtin_amdgcn_readlane(tv, l * 8 + c) & -((qv >> c) & 1);
            int sh = __builtin_amdgcn_update_dpp(0, qv, 0x111, 0xF, 0xF, true);  // row_shr:1, q_{m-1}
            sh = m ? sh : 0;
            qv = l == i ? qv : (sh ^ pr);
        }
        int lw = 0;  // log w_i = sum_{l != i} log (a_i + a_l)
#pragma unroll
        for (int l = 0; l < E; ++l)
            lw += glog[l != i ? (ai ^ A[l]) : 1];
        coef = (i < E && m < E && qv) ? gexp[(glog[qv] + 255 * 2 - lw % 255) % 255] : 0;
    };
    uint32_t acc[E][8];
#pragma unroll
    for (int r = 0; r < E; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q)
            acc[r][q] = 0;
    [&]<int... Gs>(std::integer_sequence<int, Gs...>) {
        ((wave == Gs ? syn_group<decltype(solve_rows)&, K, E, SPL, Gs>(a, emask, loff, acc, Pw, solve_rows) : void()),
         ...);
    }(std::make_integer_sequence<int, SPL>{});
    if (blockIdx.x == 0 && threadIdx.x == 0)
        a.status[b] = 0;
#pragma unroll
    for (int r = 0; r < E; ++r)
#pragma unroll
        for (int q = 0; q < 8; ++q)
            atomicXor(&syn[r * 8 + q][lane], acc[r][q]);  // ds_xor_b32, no return
    __syncthreads();
    if (!inb)
        return;
    // wave w's output rows r = w, w + SPL, ...: out_r = sum_p c[r][p] s_p,
    // each syndrome s_p already the sum of the waves' partials
    const uint32_t m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);
    for (int r = wave; r < E; r += SPL) {
        uint32_t o[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int p = 0; p < E; ++p) {
            uint32_t sy[8];
#pragma unroll
            for (int q = 0; q < 8; ++q)
                sy[q] = syn[p * 8 + q][lane];
            uint32_t x = (uint32_t)__builtin_amdgcn_readlane(coef, 8 * r + p);  // c, then c 2^a
#pragma unroll
            for (int ab = 0; ab < 8; ++ab) {
#pragma unroll
                for (int bb = 0; bb < 8; ++bb)
                    o[bb] = __builtin_amdgcn_bitop3_b32(o[bb], sy[ab], 0u - ((x >> bb) & 1u), 0x78);
                x = ((x << 1) ^ ((x & 0x80u) ? 0x1Du : 0u)) & 0xFFu;
            }
        }
        tr8(o, m4, m2, m1);
        store32(a.out + ((size_t)b * E + r) * a.pitch, off, o);
    }
}

template <int K, int E>
hipError_t launch_syn(const SynArgs& a, long long blocks, hipStream_t st)
{
    dim3 grid((unsigned)((a.len + 2047) / 2048), (unsigned)blocks);
    hipLaunchKernelGGL((k_rs_syn_split<K, E, 4>), grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

template <int K, int E, int C, int NW>
hipError_t launch(const uint8_t* src, uint8_t* out, long long pitch, long long len,
                  long long blocks, hipStream_t st, int prio)
{
    // short rows whose last tile is partial: tiles over the rows of all
    // blocks end to end (tile_pos).  A lane addresses its rows from the
    // tile's first block with a 32-bit offset (glds32's voffset): db * K *
    // pitch + o, db <= 2048 / len + 1, must stay below 2^32
    const bool flat = blocks > 1 && len % 2048 != 0 && len < 65536 && pitch % 32 == 0 &&
                      (unsigned long long)(2048 / len + 2) * K * (unsigned long long)pitch < (1ull << 32);
    Args a{src, out, pitch, len, blocks, flat ? 1 : 0, prio};
    dim3 grid(flat ? (unsigned)((blocks * len + 2047) / 2048) : (unsigned)((len + 2047) / 2048),
              flat ? 1u : (unsigned)blocks);
    if (prio)
        hipLaunchKernelGGL((k_rs_bs<K, E, C, NW, true>), grid, dim3(64 * NW), 0, st, a);
    else
        hipLaunchKernelGGL((k_rs_bs<K, E, C, NW, false>), grid, dim3(64 * NW), 0, st, a);
    return hipGetLastError();
}

RSGPU_DIAG_READER(diag_read_bs)

}  // namespace bs

bool rs_bitsliced_available(int k, int e)
{
    return (k == 16 && e == 4) || (k == 16 && e == 8) || (k == 64 && e == 32) ||
           (k == 100 && e == 20) || (k == 5 && e == 4) || (k == 20 && e == 7) ||
           (k == 64 && e == 16);
}

int rs_bitsliced_rows_per_wave(int k, int e)
{
    // (E + NW - 1) / NW of launch_rs_bitsliced's plans
    if (!rs_bitsliced_available(k, e))
        return 0;
    const int nw = (k == 64 && e == 32) || (k == 100 && e == 20) ? 4 : (k == 64 && e == 16) ? 2 : 1;
    return (e + nw - 1) / nw;
}

bool rs_bitsliced_split_available(int k, int e)
{
    return (k == 16 && e == 4) || (k == 16 && e == 8) || (k == 5 && e == 4) || (k == 20 && e == 7);
}

hipError_t launch_rs_bitsliced_split(int k, int e, const uint8_t* src, uint8_t* out, long long pitch,
                                     long long len, long long blocks, hipStream_t st)
{
    if (k == 16 && e == 4) return bs::launch_split<16, 4>(src, out, pitch, len, blocks, st);
    if (k == 16 && e == 8) return bs::launch_split<16, 8>(src, out, pitch, len, blocks, st);
    if (k == 5 && e == 4) return bs::launch_split<5, 4>(src, out, pitch, len, blocks, st);
    if (k == 20 && e == 7) return bs::launch_split<20, 7>(src, out, pitch, len, blocks, st);
    return hipErrorInvalidValue;
}

hipError_t launch_rs_syn_split(int k, int e, const SynArgs& a, long long blocks, hipStream_t st)
{
    if (blocks <= 0 || blocks > 65535 || a.len <= 0 || a.len % 32 != 0 || !a.src || !a.par || !a.out || !a.err ||
        !a.status)
        return hipErrorInvalidValue;
    if (k == 16 && e == 4) return bs::launch_syn<16, 4>(a, blocks, st);
    if (k == 16 && e == 8) return bs::launch_syn<16, 8>(a, blocks, st);
    if (k == 5 && e == 4) return bs::launch_syn<5, 4>(a, blocks, st);
    if (k == 20 && e == 7) return bs::launch_syn<20, 7>(a, blocks, st);
    return hipErrorInvalidValue;
}

hipError_t launch_rs_bitsliced(int k, int e, const uint8_t* src, uint8_t* out, long long pitch,
                               long long len, long long blocks, hipStream_t st, int prio)
{
    if (k == 16 && e == 4) return bs::launch<16, 4, 16, 1>(src, out, pitch, len, blocks, st, prio);
    if (k == 16 && e == 8) return bs::launch<16, 8, 16, 1>(src, out, pitch, len, blocks, st, prio);
    if (k == 64 && e == 32) return bs::launch<64, 32, 16, 4>(src, out, pitch, len, blocks, st, prio);
    if (k == 64 && e == 16) return bs::launch<64, 16, 16, 2>(src, out, pitch, len, blocks, st, prio);
    if (k == 100 && e == 20) return bs::launch<100, 20, 20, 4>(src, out, pitch, len, blocks, st, prio);
    if (k == 5 && e == 4) return bs::launch<5, 4, 5, 1>(src, out, pitch, len, blocks, st, prio);
    if (k == 20 && e == 7) return bs::launch<20, 7, 20, 1>(src, out, pitch, len, blocks, st, prio);
    return hipErrorInvalidValue;
}

}  // namespace rsgpu
