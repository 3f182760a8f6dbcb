// rs_kernels.hip -- MI355X (gfx950, CDNA4) kernels of the Reed-Solomon GF(2^8)
// erasure engine.  Hot path of benchmark/isa_throughput: the GF dot product
// that ISA-L computes with gf_{1..4}vect_dot_prod_avx2 (isa/gf_4vect_dot_prod_
// avx2.asm:303-451, dispatched by ec_encode_data_avx2, isa/ec_highlevel_func.c:
// 106-135) -- here as wavefront-wide byte arithmetic on the VALU.  No MFMA: the
// work is byte-wise GF(2^8) multiply-accumulate, not a float contraction.
//
// Data layout in HBM: one row per symbol, rows of a block at a fixed pitch,
// blocks back to back ([B][rows][pitch]).  A lane owns 4-byte columns of a row,
// so every wave-wide load/store is a contiguous, coalesced 256-512 B segment.
//
// Kernels
//   k_dot_generic<R>  out[r] = XOR_j c[r][j] * in[j] for RUNTIME coefficients
//                     (decode matrices, arbitrary encode matrices).  Per
//                     coefficient and dword: three v_perm_b32 8-entry lookups
//                     (bits 0-2, 3-5, 6-7 of every byte) + 1.5 v_bitop3 XORs.
//   k_rs_encode_lh<K,E> the gf_gen_rs_matrix (Vandermonde) encode with
//                     COMPILE-TIME coefficients: per source dword the 16-entry
//                     low/high nibble product tables L[n]=n*x, H[n]=(16n)*x are
//                     built in registers once (7 xtimes + 22 XORs) and every
//                     coefficient costs one v_bitop3 (acc ^= L[c&15] ^ H[c>>4]).
//   k_decode_prepare  one workgroup per block: survivor rows -> k x k matrix
//                     -> GF Gauss-Jordan inversion in LDS (isa/ec_base.c:99-152
//                     semantics, with gf_gen_decode_matrix's retry) -> decode
//                     rows (data and parity erasures) -> k_rs_tc handler
//                     addresses or v_perm tables + row pointers.
//   k_decode_prepare_syn  the closed-form decode rows of the isa_throughput
//                     case (erased originals, all parity rows surviving).
//   k_fill_synth      seeded synthetic symbols (counter-based, see rs_synth.h).
//   k_compare_rows    verify_data (isa.cpp:215-229) on the device.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <utility>

#include "gf256.h"
#include "rs_jit.h"
#include "rs_kernels.h"
#include "rs_synth.h"

namespace rsgpu {

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t vperm(uint32_t hi, uint32_t lo, uint32_t sel)
{
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// Row pointers fetched from memory are generic (flat) pointers; loads through
// them would be flat_load (out-of-order vs LDS, forcing vmcnt(0)+lgkmcnt(0)
// waits).  All rows live in global memory, so address-space-cast them.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_cu32x4;
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
__device__ __forceinline__ uint4 gload16(const uint8_t* p, long long w)
{
    const u32x4 v = ((g_cu32x4*)p)[w];
    return make_uint4(v.x, v.y, v.z, v.w);
}
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const u32x2 g_cu32x2;
typedef __attribute__((address_space(1))) u32x2 g_u32x2;
__device__ __forceinline__ uint2 gload8(const uint8_t* p, long long w)
{
    const u32x2 v = ((g_cu32x2*)p)[w];
    return make_uint2(v.x, v.y);
}
__device__ __forceinline__ void gstore8(uint8_t* p, long long w, uint2 v)
{
    u32x2 t;
    t.x = v.x; t.y = v.y;
    ((g_u32x2*)p)[w] = t;
}
__device__ __forceinline__ void gstore16(uint8_t* p, long long w, uint4 v)
{
    u32x4 t;
    t.x = v.x; t.y = v.y; t.z = v.z; t.w = v.w;
    ((g_u32x4*)p)[w] = t;
}

// ---------------------------------------------------------------------------
// Generic runtime-coefficient dot product
// ---------------------------------------------------------------------------
// Tables of one coefficient c (gf256.h perm_tables): four dwords
// {c*{0..3}, c*{4..7}, c*{0,8,16,24}, c*{32..56}} for the bits 0-2 / 3-5
// lookups (tabs4, uint4 per coefficient) and one dword c*{0,64,128,192} for
// bits 6-7 (ctab).  Layout per block: [k][rows_pad].
// srcs: [B][k] row pointers, dsts: [B][rows] row pointers (device memory).
//
// Each workgroup owns one block and a strided set of 16-byte columns; it
// stages its block's R-row slice of tabs4 in LDS once (wave-uniform
// ds_read_b128 broadcasts feed v_perm with VGPR operands, so the single
// constant-bus slot is left for the ctab dword, read with s_load).  A lane
// keeps 4 dwords x R rows of accumulators: per coefficient and dword the
// cost is three v_perm + two XORs, and one LDS broadcast per 4 dwords.

template <int R>
__global__ __launch_bounds__(256) void k_dot_generic(const uint8_t* const* __restrict__ srcs,
                                                     uint8_t* const* __restrict__ dsts,
                                                     const uint4* __restrict__ tabs4,
                                                     const uint32_t* __restrict__ ctab,
                                                     long long tab_block_stride, int k, int rows,
                                                     int rows_pad, int row0, long long n_qw,
                                                     const int* __restrict__ status)
{
    extern __shared__ uint4 ltab[];  // [k][R]
    const int b = blockIdx.y;
    if (status != nullptr && status[b] != 0)
        return;
    const uint8_t* const* S = srcs + (size_t)b * k;
    uint8_t* const* Dst = dsts + (size_t)b * rows;
    const uint4* T4 = tabs4 + (size_t)b * tab_block_stride;
    const uint32_t* TC = ctab + (size_t)b * tab_block_stride + row0;
    const int nr = (rows - row0) < R ? (rows - row0) : R;

    for (int idx = threadIdx.x; idx < k * R; idx += blockDim.x) {
        const int j = idx / R, r = idx - j * R;
        ltab[idx] = T4[(size_t)j * rows_pad + row0 + r];
    }
    __syncthreads();

    for (long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x; w < n_qw;
         w += (long long)gridDim.x * blockDim.x) {
        uint32_t acc0[R], acc1[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            acc0[r] = 0;
            acc1[r] = 0;
        }
        // two sources per step: the six lookups of a (row, dword) pair fold
        // into the accumulator with three 3-input XORs
        uint2 xa = gload8(S[0], w);
        uint2 xb = k > 1 ? gload8(S[1], w) : make_uint2(0, 0);
        int j = 0;
        for (; j + 1 < k; j += 2) {
            const uint2 a = xa, bb = xb;
            if (j + 2 < k)
                xa = gload8(S[j + 2], w);
            if (j + 3 < k)
                xb = gload8(S[j + 3], w);
            const uint32_t a00 = a.x & 0x07070707u, a01 = (a.x >> 3) & 0x07070707u, a02 = (a.x >> 6) & 0x03030303u;
            const uint32_t a10 = a.y & 0x07070707u, a11 = (a.y >> 3) & 0x07070707u, a12 = (a.y >> 6) & 0x03030303u;
            const uint32_t b00 = bb.x & 0x07070707u, b01 = (bb.x >> 3) & 0x07070707u, b02 = (bb.x >> 6) & 0x03030303u;
            const uint32_t b10 = bb.y & 0x07070707u, b11 = (bb.y >> 3) & 0x07070707u, b12 = (bb.y >> 6) & 0x03030303u;
            const uint4* lta = ltab + j * R;
            const uint4* ltb = lta + R;
            const uint32_t* cta = TC + (size_t)j * rows_pad;
            const uint32_t* ctb = cta + rows_pad;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint4 ta = lta[r], tb = ltb[r];
                const uint32_t ca = cta[r], cb = ctb[r];
                acc0[r] = xor3(acc0[r], vperm(ta.y, ta.x, a00), vperm(ta.w, ta.z, a01));
                acc0[r] = xor3(acc0[r], vperm(ca, ca, a02), vperm(tb.y, tb.x, b00));
                acc0[r] = xor3(acc0[r], vperm(tb.w, tb.z, b01), vperm(cb, cb, b02));
                acc1[r] = xor3(acc1[r], vperm(ta.y, ta.x, a10), vperm(ta.w, ta.z, a11));
                acc1[r] = xor3(acc1[r], vperm(ca, ca, a12), vperm(tb.y, tb.x, b10));
                acc1[r] = xor3(acc1[r], vperm(tb.w, tb.z, b11), vperm(cb, cb, b12));
            }
        }
        if (j < k) {
            const uint2 a = xa;
            const uint32_t a00 = a.x & 0x07070707u, a01 = (a.x >> 3) & 0x07070707u, a02 = (a.x >> 6) & 0x03030303u;
            const uint32_t a10 = a.y & 0x07070707u, a11 = (a.y >> 3) & 0x07070707u, a12 = (a.y >> 6) & 0x03030303u;
            const uint4* lta = ltab + j * R;
            const uint32_t* cta = TC + (size_t)j * rows_pad;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint4 ta = lta[r];
                const uint32_t ca = cta[r];
                acc0[r] = xor3(acc0[r], vperm(ta.y, ta.x, a00), vperm(ta.w, ta.z, a01)) ^ vperm(ca, ca, a02);
                acc1[r] = xor3(acc1[r], vperm(ta.y, ta.x, a10), vperm(ta.w, ta.z, a11)) ^ vperm(ca, ca, a12);
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (r < nr)
                gstore8(Dst[row0 + r], w, make_uint2(acc0[r], acc1[r]));
    }
}

// Byte-granular variant for unaligned pointers or the len % 16 tail: each
// thread produces one byte with the same three lookups.
__global__ __launch_bounds__(256) void k_dot_bytes(const uint8_t* const* __restrict__ srcs,
                                                   uint8_t* const* __restrict__ dsts,
                                                   const uint4* __restrict__ tabs4,
                                                   const uint32_t* __restrict__ ctab,
                                                   long long tab_block_stride, int k, int rows,
                                                   int rows_pad, long long first, long long len,
                                                   const int* __restrict__ status)
{
    const int b = blockIdx.y;
    if (status != nullptr && status[b] != 0)
        return;
    const long long i = first + (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= len)
        return;
    const uint8_t* const* S = srcs + (size_t)b * k;
    uint8_t* const* Dst = dsts + (size_t)b * rows;
    const uint4* T4 = tabs4 + (size_t)b * tab_block_stride;
    const uint32_t* TC = ctab + (size_t)b * tab_block_stride;
    for (int r = 0; r < rows; ++r) {
        uint32_t acc = 0;
        for (int j = 0; j < k; ++j) {
            const uint32_t x = S[j][i];
            const uint4 t = T4[(size_t)j * rows_pad + r];
            const uint32_t c = TC[(size_t)j * rows_pad + r];
            acc ^= vperm(t.y, t.x, x & 7u) ^ vperm(t.w, t.z, (x >> 3) & 7u) ^ vperm(c, c, (x >> 6) & 3u);
        }
        Dst[r][i] = (uint8_t)acc;
    }
}

// ---------------------------------------------------------------------------
// Compile-time-coefficient RS (gf_gen_rs_matrix) encode
// ---------------------------------------------------------------------------

template <int K, int E>
struct VandCoefs {
    uint8_t c[E][K];
    // same recurrence as gf_gen_rs_matrix (isa/ec_base.c:71-78)
    constexpr VandCoefs() : c()
    {
        uint8_t gen = 1;
        for (int p = 0; p < E; ++p) {
            uint8_t v = 1;
            for (int j = 0; j < K; ++j) {
                c[p][j] = v;
                v = gf_mul_slow(v, gen);
            }
            gen = gf_mul_slow(gen, 2);
        }
    }
};

// x * 2 for the four bytes of a dword: shift, then fold the carried-out top
// bits back in as 0x1D.  The fold multiply runs in 16-bit lanes
// (v_pk_mul_lo_u16): each half holds two flag bits 8 apart, so 0x1D*flag
// never carries across a byte.
__device__ __forceinline__ uint32_t xtime4(uint32_t x)
{
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const uint32_t hi7 = (x >> 7) & 0x01010101u;
    us2 h = __builtin_bit_cast(us2, hi7);
    h = h * (us2){0x1d, 0x1d};
    const uint32_t red = __builtin_bit_cast(uint32_t, h);
    return ((x << 1) & 0xfefefefeu) ^ red;
}

template <int K, int E>
struct VandHolder {
    static constexpr VandCoefs<K, E> v{};
};

// acc ^= c*x from the nibble tables, c a compile-time constant
template <int C>
__device__ __forceinline__ void lh_mac(uint32_t& acc, const uint32_t (&Lt)[16],
                                       const uint32_t (&Ht)[16])
{
    constexpr int lo = C & 15, hi = C >> 4;
    if constexpr (lo != 0 && hi != 0)
        acc = xor3(acc, Lt[lo], Ht[hi]);
    else if constexpr (lo != 0)
        acc ^= Lt[lo];
    else if constexpr (hi != 0)
        acc ^= Ht[hi];
}

template <int K, int E, int J, int... Rs>
__device__ __forceinline__ void lh_rows(uint32_t (&acc)[E], const uint32_t (&Lt)[16],
                                        const uint32_t (&Ht)[16],
                                        std::integer_sequence<int, Rs...>)
{
    (lh_mac<VandHolder<K, E>::v.c[Rs][J]>(acc[Rs], Lt, Ht), ...);
}

// One source row J: build L/H for this dword, fold into all E parities.
template <int K, int E, int J>
__device__ __forceinline__ void lh_source(uint32_t (&acc)[E], uint32_t x)
{
    uint32_t bs[8];
    bs[0] = x;
#pragma unroll
    for (int t = 1; t < 8; ++t)
        bs[t] = xtime4(bs[t - 1]);
    uint32_t Lt[16], Ht[16];
    Lt[0] = 0;
    Ht[0] = 0;
#pragma unroll
    for (int n = 1; n < 16; ++n) {
        const int low = n & -n;
        const int bit = low == 1 ? 0 : low == 2 ? 1 : low == 4 ? 2 : 3;
        Lt[n] = (n == low) ? bs[bit] : (Lt[n ^ low] ^ bs[bit]);
        Ht[n] = (n == low) ? bs[4 + bit] : (Ht[n ^ low] ^ bs[4 + bit]);
    }
    lh_rows<K, E, J>(acc, Lt, Ht, std::make_integer_sequence<int, E>{});
}

template <int K, int E, int J>
__device__ __forceinline__ void lh_sources(uint32_t (&acc)[E], const uint8_t* sb, long long pitch,
                                           long long w, uint32_t x)
{
    uint32_t xn = 0;
    if constexpr (J + 1 < K)
        xn = reinterpret_cast<const uint32_t*>(sb + (size_t)(J + 1) * pitch)[w];
    lh_source<K, E, J>(acc, x);
    if constexpr (J + 1 < K)
        lh_sources<K, E, J + 1>(acc, sb, pitch, w, xn);
}

template <int K, int E>
__global__ __launch_bounds__(256) void k_rs_encode_lh(const uint8_t* __restrict__ src,
                                                      uint8_t* __restrict__ par, long long pitch,
                                                      long long n_dw)
{
    const int b = blockIdx.y;
    const uint8_t* sb = src + (size_t)b * K * pitch;
    uint8_t* pb = par + (size_t)b * E * pitch;

    for (long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x; w < n_dw;
         w += (long long)gridDim.x * blockDim.x) {
        uint32_t acc[E];
#pragma unroll
        for (int r = 0; r < E; ++r)
            acc[r] = 0;
        const uint32_t x0 = reinterpret_cast<const uint32_t*>(sb)[w];
        lh_sources<K, E, 0>(acc, sb, pitch, w, x0);
#pragma unroll
        for (int r = 0; r < E; ++r)
            reinterpret_cast<uint32_t*>(pb + (size_t)r * pitch)[w] = acc[r];
    }
}

// ---------------------------------------------------------------------------
// Decode preparation: one workgroup per block (PrepArgs, rs_kernels.h)
// ---------------------------------------------------------------------------
// Per block: status (0; -1 singular, "BAD MATRIX"; -2 malformed erasure
// list), survivor row pointers [k], output row pointers [nerrs], and the
// decode rows as k_rs_tc handler addresses (pass layout) or v_perm tables
// [k][rows_pad][5].  LDS: log / antilog, the erasure flags, the survivor
// list and two k x k byte matrices.

// log / antilog tables of GF(2^8), a compile-time constant (gf256.h)
__device__ const GfTables kGfTables = make_gf_tables();

__global__ __launch_bounds__(256) void k_decode_prepare(PrepArgs a)
{
    extern __shared__ __align__(16) uint8_t lds[];
    uint8_t* gexp = lds;             // 512
    uint8_t* glog = lds + 512;       // 256
    uint8_t* in_err = lds + 768;     // 256
    uint8_t* surv = lds + 1024;      // 256: decode_index (erasure_code_base_test.c:156-162)
    int* sh = reinterpret_cast<int*>(lds + 1280);  // 16 ints
    const int k = a.k, m = a.m, ne = a.nerrs;
    uint8_t* A = lds + 1344;         // k*k
    uint8_t* Dm = A + k * k;         // k*k

    const int b = blockIdx.x;
    const int tid = threadIdx.x, nt = blockDim.x;
    const uint8_t* eb = a.err + (size_t)b * ne;

    for (int i = tid; i < 512; i += nt) {
        gexp[i] = kGfTables.exp[i];
        if (i < 256)
            glog[i] = kGfTables.log[i];
    }
    for (int i = tid; i < 256; i += nt)
        in_err[i] = 0;
    __syncthreads();
    if (tid == 0) {
        // validate: strictly ascending, < m (< k for the isa_decoder form),
        // at most m - k erasures (k survivors must exist)
        int bad = ne > m - k;
        int nsrc = 0;
        for (int i = 0; i < ne; ++i) {
            const int j = eb[i];
            bad |= j >= m || (a.originals_only && j >= k) || (i > 0 && j <= eb[i - 1]);
            nsrc += j < k;
        }
        if (!bad) {
            for (int i = 0; i < ne; ++i)
                in_err[eb[i]] = 1;
            // survivors: the first k rows not erased, ascending (isa.cpp:177-
            // 182; erasure_code_base_test.c:156-162)
            int r = 0;
            for (int i = 0; i < k; ++i, ++r) {
                while (in_err[r])
                    ++r;
                surv[i] = (uint8_t)r;
            }
        }
        sh[0] = bad ? -2 : 0;
        sh[2] = nsrc;  // nsrcerrs: the data erasures come first (ascending)
        sh[3] = 0;     // incr of the retry loop
    }
    __syncthreads();
    if (sh[0] != 0) {
        if (tid == 0)
            a.status[b] = sh[0];
        return;
    }
    auto gmul = [&](uint8_t x, uint8_t y) -> uint8_t {
        return (x && y) ? gexp[glog[x] + glog[y]] : (uint8_t)0;
    };
    // encode-matrix entry (row r, column j): the caller's matrix, or
    // gf_gen_rs_matrix (isa/ec_base.c:62-79: identity, then 2^(p j))
    auto enc = [&](int r, int j) -> uint8_t {
        if (a.enc)
            return a.enc[(size_t)r * k + j];
        if (r < k)
            return r == j ? 1 : 0;
        return gexp[((r - k) * j) % 255];
    };
    for (;;) {
        // b[i][j] = encode row surv[i]
        for (int idx = tid; idx < k * k; idx += nt) {
            const int i = idx / k, j = idx - i * k;
            A[idx] = enc(surv[i], j);
            Dm[idx] = (i == j) ? 1 : 0;
        }
        __syncthreads();
        // Gauss-Jordan (isa/ec_base.c:99-152): zero pivot -> swap with the
        // first lower row holding a non-zero in that column; singular -> -1
        int singular = 0;
        for (int i = 0; i < k; ++i) {
            if (tid == 0) {
                int piv = i;
                if (A[i * k + i] == 0) {
                    piv = -1;
                    for (int j = i + 1; j < k; ++j)
                        if (A[j * k + i]) {
                            piv = j;
                            break;
                        }
                }
                sh[1] = piv;
            }
            __syncthreads();
            const int piv = sh[1];
            if (piv < 0) {
                singular = 1;
                break;
            }
            if (piv != i) {
                for (int c = tid; c < k; c += nt) {
                    uint8_t t = A[i * k + c];
                    A[i * k + c] = A[piv * k + c];
                    A[piv * k + c] = t;
                    t = Dm[i * k + c];
                    Dm[i * k + c] = Dm[piv * k + c];
                    Dm[piv * k + c] = t;
                }
                __syncthreads();
            }
            const uint8_t pinv = gexp[255 - glog[A[i * k + i]]];
            __syncthreads();
            for (int c = tid; c < k; c += nt) {
                A[i * k + c] = gmul(A[i * k + c], pinv);
                Dm[i * k + c] = gmul(Dm[i * k + c], pinv);
            }
            __syncthreads();
            // eliminate column i from every other row; factor read before update
            for (int idx = tid; idx < k * k; idx += nt) {
                const int r = idx / k, c = idx - r * k;
                if (r == i || c == i)
                    continue;  // column i updated after the sweep
                const uint8_t f = A[r * k + i];
                A[idx] ^= gmul(f, A[i * k + c]);
                Dm[idx] ^= gmul(f, Dm[i * k + c]);
            }
            __syncthreads();
            for (int r = tid; r < k; r += nt) {
                if (r == i)
                    continue;
                const uint8_t f = A[r * k + i];
                // column i of Dm was handled in the sweep only for c != i
                Dm[r * k + i] ^= gmul(f, Dm[i * k + i]);
                A[r * k + i] = 0;
            }
            __syncthreads();
        }
        if (!singular)
            break;
        // the reference's retry (erasure_code_base_test.c:163-184): with all
        // m - k rows erased there is nothing to swap in ("BAD MATRIX");
        // otherwise the last survivor moves `incr` rows further, stepping
        // over erased parity rows listed in src_err_list[nsrcerrs ..
        // nerrs - nsrcerrs) (the loop bound as written there)
        if (tid == 0) {
            int st = 0;
            if (ne == m - k) {
                st = -1;
            } else {
                int incr = sh[3] + 1;
                const int nsrc = sh[2];
                for (int i = nsrc; i < ne - nsrc; ++i)
                    if (eb[i] == surv[k - 1] + incr)
                        ++incr;
                if (surv[k - 1] + incr >= m)
                    st = -1;
                else
                    surv[k - 1] = (uint8_t)(surv[k - 1] + incr);
                sh[3] = incr;
            }
            sh[0] = st;
        }
        __syncthreads();
        if (sh[0] != 0)
            break;
    }
    __syncthreads();
    const int st = sh[0];
    if (tid == 0)
        a.status[b] = st;
    if (st != 0)
        return;
    // pointers: survivors from the data / parity rows, outputs
    for (int i = tid; i < k; i += nt) {
        const int r = surv[i];
        a.surv_ptrs[(size_t)b * k + i] = (r < k) ? a.src + ((size_t)b * k + r) * a.src_pitch
                                                 : a.par + ((size_t)b * (m - k) + (r - k)) * a.par_pitch;
    }
    for (int i = tid; i < ne; i += nt)
        a.out_ptrs[(size_t)b * ne + i] = a.out + ((size_t)b * ne + i) * a.out_pitch;
    // decode row i, survivor column j (erasure_code_base_test.c:197-210;
    // isa.cpp:200-204): data erasures take row err[i] of inv(b); parity
    // erasures the encode row times inv(b)
    const int nsrc = sh[2];
    auto coef = [&](int i, int j) -> uint8_t {
        if (i < nsrc)
            return Dm[eb[i] * k + j];
        const int r = eb[i];
        uint8_t s = 0;
        for (int q = 0; q < k; ++q)
            s ^= gmul(Dm[q * k + j], enc(r, q));
        return s;
    };
    if (a.coef_out) {
        uint8_t* cb = a.coef_out + (size_t)b * ne * k;
        for (int idx = tid; idx < ne * k; idx += nt) {
            const int i = idx / k, j = idx - i * k;
            cb[idx] = coef(i, j);
        }
        return;
    }
    if (a.tc_addr && a.tc_table) {
        // k_rs_tc handler addresses (pass layout), padding slots -> handler 0
        unsigned long long* ta = a.tc_addr + (size_t)b * a.tc_block_stride;
        const int np = tc_passes(ne);
        for (int p = 0; p < np; ++p) {
            const int pr = tc_pass_rows(ne, p), slots = tc_rows_per_pass(pr);
            unsigned long long* tp = ta + tc_pass_offset(k, p);
            for (int idx = tid; idx < k * slots; idx += nt) {
                const int j = idx / slots, s = idx - j * slots;
                tp[idx] = a.tc_table[(s & 7) * 256 + (s < pr ? coef(32 * p + s, j) : 0)];
            }
        }
        return;
    }
    // v_perm tables: [j][rows_pad], rows beyond nerrs zero
    uint4* t4 = a.tabs4 + (size_t)b * a.tab_block_stride;
    uint32_t* tc = a.ctab + (size_t)b * a.tab_block_stride;
    const int rows_pad = a.rows_pad;
    for (int idx = tid; idx < k * rows_pad; idx += nt) {
        const int j = idx / rows_pad, r = idx - j * rows_pad;
        uint32_t t[5] = {0, 0, 0, 0, 0};
        if (r < ne) {
            const uint8_t c = coef(r, j);
            uint8_t v[20];
#pragma unroll
            for (int n = 0; n < 8; ++n) {
                v[n] = gmul(c, (uint8_t)n);
                v[8 + n] = gmul(c, (uint8_t)(n << 3));
            }
#pragma unroll
            for (int n = 0; n < 4; ++n)
                v[16 + n] = gmul(c, (uint8_t)(n << 6));
#pragma unroll
            for (int q = 0; q < 5; ++q)
                t[q] = (uint32_t)v[4 * q] | ((uint32_t)v[4 * q + 1] << 8) |
                       ((uint32_t)v[4 * q + 2] << 16) | ((uint32_t)v[4 * q + 3] << 24);
        }
        t4[idx] = make_uint4(t[0], t[1], t[2], t[3]);
        tc[idx] = t[4];
    }
}

// ---------------------------------------------------------------------------
// Synthetic data and verification
// ---------------------------------------------------------------------------

// Rows over the grid's y dimension (grid-stride), 8-byte words over x: no
// per-element 64-bit division (a flat index split by a runtime row length
// cost ~130 VALU per word; the fill of a C4 batch took ~25 ms).
__global__ __launch_bounds__(256) void k_fill_synth(uint8_t* __restrict__ dst, long long rows,
                                                    long long len, long long pitch,
                                                    unsigned long long seed,
                                                    unsigned long long row0)
{
    const long long words = (len + 7) / 8;
    const bool whole = (pitch % 8) == 0 && (reinterpret_cast<uintptr_t>(dst) & 7) == 0;
    for (long long r = blockIdx.y; r < rows; r += gridDim.y) {
        uint8_t* row = dst + r * pitch;
        for (long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x; w < words;
             w += (long long)gridDim.x * blockDim.x) {
            const uint64_t v = synth_word(seed, row0 + (uint64_t)r, (uint64_t)w);
            uint8_t* p = row + w * 8;
            if (whole && w * 8 + 8 <= len) {
                *reinterpret_cast<uint64_t*>(p) = v;
            } else {
                for (int q = 0; q < 8 && w * 8 + q < len; ++q)
                    p[q] = (uint8_t)(v >> (8 * q));
            }
        }
    }
}

// mismatches[b] += number of differing bytes between recovered row i of block
// b and the original row err[b][i] of that block.
__global__ __launch_bounds__(256) void k_compare_rows(const uint8_t* __restrict__ src,
                                                      long long src_pitch, int k,
                                                      const uint8_t* __restrict__ out,
                                                      long long out_pitch, int e,
                                                      const uint8_t* __restrict__ err,
                                                      long long len,
                                                      unsigned long long* __restrict__ mismatches)
{
    const int b = blockIdx.z, i = blockIdx.y;
    const uint8_t* o = out + ((size_t)b * e + i) * out_pitch;
    const int sidx = err[(size_t)b * e + i];
    if (sidx >= k) {  // not an original: count the whole row as unverifiable
        if (blockIdx.x == 0 && threadIdx.x == 0)
            atomicAdd(&mismatches[b], (unsigned long long)len);
        return;
    }
    const uint8_t* s = src + ((size_t)b * k + sidx) * src_pitch;
    unsigned long long bad = 0;
    long long head = 0;  // bytes compared 16 at a time
    if (((reinterpret_cast<uintptr_t>(o) | reinterpret_cast<uintptr_t>(s)) & 15) == 0) {
        head = len & ~15LL;
        for (long long p = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 16; p < head;
             p += (long long)gridDim.x * blockDim.x * 16) {
            const uint4 x = *reinterpret_cast<const uint4*>(o + p);
            const uint4 y = *reinterpret_cast<const uint4*>(s + p);
            const uint32_t d[4] = {x.x ^ y.x, x.y ^ y.y, x.z ^ y.z, x.w ^ y.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // differing bytes: a bit per nonzero byte of d
                uint32_t t = d[q] | (d[q] >> 4);
                t |= t >> 2;
                t |= t >> 1;
                bad += __builtin_popcount(t & 0x01010101u);
            }
        }
    }
    for (long long p = head + (long long)blockIdx.x * blockDim.x + threadIdx.x; p < len;
         p += (long long)gridDim.x * blockDim.x)
        bad += (o[p] != s[p]);
    // wave reduction then one atomic per wave
    for (int off = 32; off > 0; off >>= 1)
        bad += __shfl_down(bad, off, 64);
    if ((threadIdx.x & 63) == 0 && bad)
        atomicAdd(&mismatches[b], bad);
}

// ---------------------------------------------------------------------------
// Host launch wrappers (declared in rs_kernels.h)
// ---------------------------------------------------------------------------

template <int R>
static hipError_t launch_generic_R(const DotArgs& a, hipStream_t st)
{
    const long long n_ow = a.len / 8;  // 8-byte words per lane
    if (n_ow > 0) {
        const size_t lds = (size_t)a.k * R * sizeof(uint4);
        static bool attr_set = false;
        if (!attr_set) {
            (void)hipFuncSetAttribute((const void*)k_dot_generic<R>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr_set = true;
        }
        long long per_block = (n_ow + 255) / 256;
        long long fill = (2048 + a.blocks - 1) / a.blocks;
        long long gx = per_block < fill ? per_block : fill;
        if (gx < 1)
            gx = 1;
        dim3 grid((unsigned)gx, (unsigned)a.blocks);
        for (int row0 = 0; row0 < a.rows; row0 += R) {
            hipLaunchKernelGGL(k_dot_generic<R>, grid, dim3(256), lds, st, a.srcs, a.dsts, a.tabs4,
                               a.ctab, a.tab_block_stride, a.k, a.rows, a.rows_pad, row0, n_ow,
                               a.status);
        }
    }
    const long long first = n_ow * 8;
    if (first < a.len) {
        const long long nb = a.len - first;
        dim3 grid((unsigned)((nb + 255) / 256), (unsigned)a.blocks);
        hipLaunchKernelGGL(k_dot_bytes, grid, dim3(256), 0, st, a.srcs, a.dsts, a.tabs4, a.ctab,
                           a.tab_block_stride, a.k, a.rows, a.rows_pad, first, a.len, a.status);
    }
    return hipGetLastError();
}

int generic_rows_per_pass(int rows)
{
    static const int Rs[] = {1, 2, 4, 8, 12, 16, 20, 24, 32};
    const int want = rows < 32 ? rows : 32;
    for (int r : Rs)
        if (r >= want)
            return r;
    return 32;
}

hipError_t launch_dot_generic(const DotArgs& a, hipStream_t st)
{
    if (a.bytewise) {
        dim3 grid((unsigned)((a.len + 255) / 256), (unsigned)a.blocks);
        hipLaunchKernelGGL(k_dot_bytes, grid, dim3(256), 0, st, a.srcs, a.dsts, a.tabs4, a.ctab,
                           a.tab_block_stride, a.k, a.rows, a.rows_pad, 0LL, a.len, a.status);
        return hipGetLastError();
    }
    switch (generic_rows_per_pass(a.rows)) {
    case 1: return launch_generic_R<1>(a, st);
    case 2: return launch_generic_R<2>(a, st);
    case 4: return launch_generic_R<4>(a, st);
    case 8: return launch_generic_R<8>(a, st);
    case 12: return launch_generic_R<12>(a, st);
    case 16: return launch_generic_R<16>(a, st);
    case 20: return launch_generic_R<20>(a, st);
    case 24: return launch_generic_R<24>(a, st);
    default: return launch_generic_R<32>(a, st);
    }
}

template <int K, int E>
static hipError_t launch_lh(const uint8_t* src, uint8_t* par, long long pitch, long long len,
                            long long blocks, hipStream_t st)
{
    const long long n_dw = len / 4;
    const long long want = (n_dw + 255) / 256;
    const long long cap = 65535;
    dim3 grid((unsigned)(want < cap ? want : cap), (unsigned)blocks);
    hipLaunchKernelGGL((k_rs_encode_lh<K, E>), grid, dim3(256), 0, st, src, par, pitch, n_dw);
    return hipGetLastError();
}

bool rs_encode_specialized_available(int k, int e)
{
    return (k == 16 && e == 4) || (k == 16 && e == 8) || (k == 64 && e == 32) ||
           (k == 100 && e == 20) || (k == 5 && e == 4);
}

hipError_t launch_rs_encode_specialized(int k, int e, const uint8_t* src, uint8_t* par,
                                        long long pitch, long long len, long long blocks,
                                        hipStream_t st)
{
    if (k == 16 && e == 4) return launch_lh<16, 4>(src, par, pitch, len, blocks, st);
    if (k == 16 && e == 8) return launch_lh<16, 8>(src, par, pitch, len, blocks, st);
    if (k == 64 && e == 32) return launch_lh<64, 32>(src, par, pitch, len, blocks, st);
    if (k == 100 && e == 20) return launch_lh<100, 20>(src, par, pitch, len, blocks, st);
    if (k == 5 && e == 4) return launch_lh<5, 4>(src, par, pitch, len, blocks, st);
    return hipErrorInvalidValue;
}

size_t decode_prepare_lds_bytes(int k) { return 1344 + 2 * (size_t)k * k; }

hipError_t launch_decode_prepare(const PrepArgs& a, hipStream_t st)
{
    if (a.k <= 0 || a.k > 250 || a.m < a.k || a.m > 256 || a.nerrs <= 0)
        return hipErrorInvalidValue;
    const size_t lds = decode_prepare_lds_bytes(a.k);
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_decode_prepare,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(k_decode_prepare, dim3((unsigned)a.blocks), dim3(256), lds, st, a);
    return hipGetLastError();
}

hipError_t launch_fill_synth(uint8_t* dst, long long rows, long long len, long long pitch,
                             unsigned long long seed, unsigned long long row0, hipStream_t st)
{
    const long long words = (len + 7) / 8;
    if (rows <= 0 || words <= 0)
        return hipSuccess;
    const long long gx = std::min<long long>((words + 255) / 256, 1024);
    const long long gy = std::min<long long>(rows, 65535);
    hipLaunchKernelGGL(k_fill_synth, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, st, dst, rows, len,
                       pitch, seed, row0);
    return hipGetLastError();
}

hipError_t launch_compare_rows(const uint8_t* src, long long src_pitch, int k, const uint8_t* out,
                               long long out_pitch, int e, const uint8_t* err, long long len,
                               long long blocks, unsigned long long* mismatches, hipStream_t st)
{
    // 16 bytes per lane: 4 KB per workgroup pass
    const long long want = std::max<long long>(1, std::min<long long>((len + 4095) / 4096, 64));
    dim3 grid((unsigned)want, (unsigned)e, (unsigned)blocks);
    hipLaunchKernelGGL(k_compare_rows, grid, dim3(256), 0, st, src, src_pitch, k, out, out_pitch,
                       e, err, len, mismatches);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Row pointer tables and the single-source update (ec_encode_data_update)
// ---------------------------------------------------------------------------

// out[b][r] = base + (b*rows_per_block + r)*pitch
__global__ __launch_bounds__(256) void k_row_ptrs(const uint8_t* base, long long pitch,
                                                  int rows_per_block, long long blocks,
                                                  const uint8_t** out)
{
    const long long n = blocks * rows_per_block;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        out[i] = base + i * pitch;
}

// coding[r][i] ^= c_r * data[i]  (isa/ec_base.c:307-321 semantics); tables as
// the generic kernel: tabs4/ctab [rows] of the column vec_i.
__global__ __launch_bounds__(256) void k_update(const uint8_t* __restrict__ data,
                                                uint8_t* const* __restrict__ coding,
                                                const uint4* __restrict__ tabs4,
                                                const uint32_t* __restrict__ ctab, long long len)
{
    const int r = blockIdx.y;
    const uint4 t = tabs4[r];
    const uint32_t c = ctab[r];
    uint8_t* out = coding[r];
    const bool vec = ((reinterpret_cast<uintptr_t>(data) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    const long long n_ow = vec ? len / 16 : 0;
    for (long long w = (long long)blockIdx.x * blockDim.x + threadIdx.x; w < n_ow;
         w += (long long)gridDim.x * blockDim.x) {
        const uint4 x = gload16(data, w);
        uint4 o = gload16(out, w);
        o.x ^= vperm(t.y, t.x, x.x & 0x07070707u) ^ vperm(t.w, t.z, (x.x >> 3) & 0x07070707u) ^ vperm(c, c, (x.x >> 6) & 0x03030303u);
        o.y ^= vperm(t.y, t.x, x.y & 0x07070707u) ^ vperm(t.w, t.z, (x.y >> 3) & 0x07070707u) ^ vperm(c, c, (x.y >> 6) & 0x03030303u);
        o.z ^= vperm(t.y, t.x, x.z & 0x07070707u) ^ vperm(t.w, t.z, (x.z >> 3) & 0x07070707u) ^ vperm(c, c, (x.z >> 6) & 0x03030303u);
        o.w ^= vperm(t.y, t.x, x.w & 0x07070707u) ^ vperm(t.w, t.z, (x.w >> 3) & 0x07070707u) ^ vperm(c, c, (x.w >> 6) & 0x03030303u);
        gstore16(out, w, o);
    }
    for (long long i = n_ow * 16 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < len;
         i += (long long)gridDim.x * blockDim.x) {
        const uint32_t x = data[i];
        out[i] ^= (uint8_t)(vperm(t.y, t.x, x & 7u) ^ vperm(t.w, t.z, (x >> 3) & 7u) ^ vperm(c, c, (x >> 6) & 3u));
    }
}

hipError_t launch_row_ptrs(const uint8_t* base, long long pitch, int rows_per_block,
                           long long blocks, const uint8_t** out, hipStream_t st)
{
    long long n = blocks * rows_per_block;
    long long g = (n + 255) / 256;
    if (g > 4096)
        g = 4096;
    if (g < 1)
        g = 1;
    hipLaunchKernelGGL(k_row_ptrs, dim3((unsigned)g), dim3(256), 0, st, base, pitch,
                       rows_per_block, blocks, out);
    return hipGetLastError();
}

hipError_t launch_update(const uint8_t* data, uint8_t* const* coding, const uint4* tabs4,
                         const uint32_t* ctab, int rows, long long len, hipStream_t st)
{
    long long g = (len / 16 + 255) / 256;
    if (g > 1024)
        g = 1024;
    if (g < 1)
        g = 1;
    hipLaunchKernelGGL(k_update, dim3((unsigned)g, (unsigned)rows), dim3(256), 0, st, data,
                       coding, tabs4, ctab, len);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Decode preparation, closed form (one workgroup per block)
// ---------------------------------------------------------------------------
// With all e parity rows surviving and e erased ORIGINALS E = {j_0 < ... },
// the survivor matrix b of isa.cpp:177-182 is singular iff the e x e block
// V_E[p][i] = 2^(p*j_i) is (det b = det V_E up to row order), and V_E is
// Vandermonde in distinct points, so never singular.  The recovered symbols
// are the unique solution of V_E x = s with the syndromes
// s_p = P_p ^ sum_{j not in E} 2^(p j) d_j; the decode rows below apply
// V_E^-1 [V_kept | I] to the survivors and the parity rows in one pass.
// Outputs: srcs[b][k] (survivors ascending, then the parity rows), dsts[b][e]
// = out rows, status, and either the k_rs_tc handler addresses dir_addr
// [b][k][slots] or the decode rows jit_coef [b][e][k] for the emitters.
__global__ __launch_bounds__(256) void k_decode_prepare_syn(int k, int e,
                                                            const uint8_t* __restrict__ err,
                                                            uint8_t* out, long long out_pitch,
                                                            const uint8_t** srcs, uint8_t** dsts,
                                                            const unsigned long long* tc_table,
                                                            int* status, const uint8_t* src,
                                                            const uint8_t* par,
                                                            unsigned long long* dir_addr,
                                                            uint8_t* jit_coef)
{
    extern __shared__ __align__(16) uint8_t lds[];
    uint8_t* gexp = lds;          // 512
    uint8_t* glog = lds + 512;    // 256
    int* sh = reinterpret_cast<int*>(lds + 768);  // 16 ints
    uint8_t* A = lds + 832;       // e*e
    const int b = blockIdx.x;
    const int tid = threadIdx.x, nt = blockDim.x;
    const uint8_t* eb = err + (size_t)b * e;
    uint8_t* lv = A + e * e;   // survivors, k - e bytes (256 reserved)
    uint8_t* lam = lv + 256;   // Lambda coefficients, e + 1 (128 reserved)
    uint8_t* lw = lam + 128;   // log w_i (128 reserved)
    uint8_t* lb = lw + 128;    // log Lambda(b_q) (256 reserved)
    uint8_t* ea = lb + 256;    // the erased originals j_i (128 reserved)
    uint8_t* aa = ea + 128;    // a_i = 2^(j_i) (128 reserved)
    for (int i = tid; i < 512; i += nt) {
        gexp[i] = kGfTables.exp[i];
        if (i < 256)
            glog[i] = kGfTables.log[i];
    }
    if (tid < e)  // the list once from global memory, all lanes at once
        ea[tid] = eb[tid];
    if (tid == 0)
        sh[0] = 0;
    __syncthreads();
    // validate: strictly ascending originals (one lane per entry; a serial
    // loop of dependent byte loads here was most of this kernel's time)
    if (tid < e && (ea[tid] >= k || (tid > 0 && ea[tid] <= ea[tid - 1])))
        sh[0] = -2;
    __syncthreads();
    if (sh[0] != 0) {
        if (tid == 0)
            status[b] = sh[0];
        return;
    }
    auto gmul = [&](uint8_t x, uint8_t y) -> uint8_t {
        return (x && y) ? gexp[glog[x] + glog[y]] : (uint8_t)0;
    };
    const int tc_rows = tc_rows_per_pass(e);
    {
        // One-matrix decode through k_rs_tc: sources = the k - e surviving
        // originals (ascending) then the e parity rows, outputs = the erased
        // originals.  d_E = V_E^-1 (P ^ V_kept d_kept), V_E[p][i] = a_i^p with
        // a_i = 2^(j_i) (gf_gen_rs_matrix rows k + p, isa/ec_base.c:71-78):
        // the rows of inv(b) that isa.cpp:177-209 applies (the unique
        // solution, so bit-exact with the reference's decode).  V_E is
        // Vandermonde in distinct points, so it is never singular, and both
        // blocks have closed forms (Lagrange basis L_i of the points a_l,
        // Lambda(z) = prod_l (z + a_l), w_i = prod_{l != i} (a_i + a_l)):
        //   (V_E^-1)[i][p]          = [z^p] L_i(z) = [z^p] (Lambda(z) / (z + a_i)) / w_i
        //   (V_E^-1 V_kept)[i][q]   = L_i(b_q)     = Lambda(b_q) / ((b_q + a_i) w_i)
        // with b_q = 2^(j_q) for survivor q: O(e k) work, no elimination.
        const int nl = k - e;
        for (int i = tid; i < e; i += nt)
            aa[i] = gexp[ea[i]];
        __syncthreads();
        for (int j = tid; j < k; j += nt) {
            int below = 0;  // erased originals < j (the list is validated ascending)
            bool er = false;
            for (int i = 0; i < e; ++i) {
                below += ea[i] < j;
                er |= ea[i] == j;
            }
            if (!er)
                lv[j - below] = (uint8_t)j;
        }
        if (e < 64) {
            if (tid < 64) {  // Lambda(z) by wave 0, lane m holding the coefficient of z^m
                uint8_t lm = tid == 0 ? 1 : 0;  // e + 1 <= 64 lanes
                for (int l = 0; l < e; ++l) {   // times (z + a_l): lam_m <- lam_{m-1} + a_l lam_m
                    const int below = __shfl_up((int)lm, 1);
                    lm = (uint8_t)(tid == 0 ? 0 : below) ^ gmul(aa[l], lm);
                }
                if (tid <= e)
                    lam[tid] = lm;
            }
        } else {
            // e + 1 > 64 coefficients (e <= 125): thread m <= e holds lam_m and
            // the product grows through LDS, one factor per barrier pair
            uint8_t lm = tid == 0 ? 1 : 0;
            for (int l = 0; l < e; ++l) {
                if (tid <= e)
                    lam[tid] = lm;
                __syncthreads();
                if (tid <= e)
                    lm = (uint8_t)(tid == 0 ? 0 : lam[tid - 1]) ^ gmul(aa[l], lm);
                __syncthreads();
            }
            if (tid <= e)
                lam[tid] = lm;
        }
        for (int i = tid; i < e; i += nt) {
            const uint8_t a = aa[i];
            int lg = 0;
            for (int l = 0; l < e; ++l)
                if (l != i)
                    lg += glog[a ^ aa[l]];
            lw[i] = (uint8_t)(lg % 255);
        }
        __syncthreads();
        for (int q = tid; q < nl; q += nt) {  // log Lambda(b_q) = sum_l log(b_q + a_l), never 0
            const uint8_t bq = gexp[lv[q]];
            int lg = 0;
            for (int l = 0; l < e; ++l)
                lg += glog[bq ^ aa[l]];
            lb[q] = (uint8_t)(lg % 255);
        }
        for (int i = tid; i < e; i += nt) {  // row i of V_E^-1 by synthetic division
            const uint8_t a = aa[i];
            uint8_t qm = lam[e];  // q_{e-1}
            for (int m = e - 1; m >= 0; --m) {
                A[i * e + m] = qm ? gexp[(glog[qm] + 255 - lw[i]) % 255] : (uint8_t)0;
                if (m)
                    qm = lam[m] ^ gmul(a, qm);
            }
        }
        __syncthreads();
        if (tid == 0)
            status[b] = 0;
        for (int q = tid; q < k; q += nt)
            srcs[(size_t)b * k + q] = q < nl ? src + ((size_t)b * k + lv[q]) * out_pitch
                                             : par + ((size_t)b * e + (q - nl)) * out_pitch;
        for (int i = tid; i < e; i += nt)
            dsts[(size_t)b * e + i] = out + ((size_t)b * e + i) * out_pitch;
        // decode row i, source q (survivors ascending, then the parity rows)
        auto dcoef = [&](int q, int i) -> uint8_t {
            if (i >= e)
                return 0;
            if (q < nl) {
                const uint8_t d = gexp[lv[q]] ^ aa[i];  // b_q + a_i, never 0
                return gexp[(lb[q] + 2 * 255 - glog[d] - lw[i]) % 255];
            }
            return A[i * e + (q - nl)];
        };
        if (jit_coef) {
            // k_rs_jit's decode rows [e][k] for k_jit_emit (coalesced here,
            // the code is written by one workgroup per (wave, chunk) there)
            uint8_t* cb = jit_coef + (size_t)b * e * k;
            for (int idx = tid; idx < e * k; idx += nt) {
                const int i = idx / k, q = idx - i * k;
                cb[idx] = dcoef(q, i);
            }
            return;
        }
        unsigned long long* da = dir_addr + (size_t)b * k * tc_rows;
        for (int idx = tid; idx < k * tc_rows; idx += nt) {
            const int q = idx / tc_rows, i = idx - q * tc_rows;
            da[idx] = tc_table[(i & 7) * 256 + dcoef(q, i)];
        }
    }
}

size_t decode_prepare_syn_lds_bytes(int e) { return 832 + (size_t)e * e + 1024; }

hipError_t launch_decode_prepare_syn(int k, int e, long long blocks, const uint8_t* err,
                                     uint8_t* out, long long out_pitch, const uint8_t** srcs,
                                     uint8_t** dsts, const unsigned long long* tc_table, int* status,
                                     const uint8_t* src, const uint8_t* par,
                                     unsigned long long* dir_addr, uint8_t* jit_coef, hipStream_t st)
{
    if (k <= 0 || k > 250 || e <= 0 || e > (jit_coef ? 125 : 32) || e > k || k + e > 250 ||
        (!jit_coef && (!tc_table || !dir_addr)))
        return hipErrorInvalidValue;
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_decode_prepare_syn,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    hipLaunchKernelGGL(k_decode_prepare_syn, dim3((unsigned)blocks), dim3(256),
                       decode_prepare_syn_lds_bytes(e), st, k, e, err, out, out_pitch, srcs, dsts,
                       tc_table, status, src, par, dir_addr, jit_coef);
    return hipGetLastError();
}

}  // namespace rsgpu
