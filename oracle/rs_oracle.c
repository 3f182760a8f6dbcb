/*
 * rs_oracle.c -- CPU restatement of the ISA-L 2.13 Reed-Solomon GF(2^8) path
 * exercised by benchmark/isa_throughput (TEST INFRASTRUCTURE ONLY).
 *
 * This file is the parity oracle for the MI355X engine.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product path (storage-benchmarks_amd/) never links or calls it.
 *
 * It is a restatement, not a copy: the field tables are generated at start-up
 * from the primitive polynomial instead of being transcribed, and the dot
 * product uses a per-coefficient 256-entry product row.  Every function cites
 * the reference function whose behaviour it follows (paths relative to
 * /root/reference/isa-l_open_src_2.13/).
 *
 * Pinning: tests/test_oracle.py checks this file against
 *   - the ISA-L base C compiled from the reference sources (oracle/_ref/,
 *     built by oracle/Makefile) on random inputs, and
 *   - the known-answer vectors held by the reference's own tests
 *     (erasure_code/gf_inverse_test.c:124-179, gf_vect_mul_test.c:53-80),
 *   - the committed golden fixtures in tests/golden/.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rs_oracle.h"

static uint8_t g_exp[512];
static uint8_t g_log[256];
static uint8_t g_mul[256][256];
static int g_ready = 0;

/* Field: GF(2^8), primitive polynomial x^8+x^4+x^3+x^2+1 (0x11D), generator 2.
 * ec_base.h:35 (gff_base) / :64 (gflog_base) hold the same tables verbatim;
 * here they are derived. */
void orc_init(void)
{
    if (g_ready)
        return;
    unsigned v = 1;
    for (int i = 0; i < 255; ++i) {
        g_exp[i] = (uint8_t)v;
        g_exp[i + 255] = (uint8_t)v;
        g_log[v] = (uint8_t)i;
        v <<= 1;
        if (v & 0x100)
            v ^= 0x11D;
    }
    g_exp[510] = g_exp[0];
    g_exp[511] = g_exp[1];
    g_log[0] = 0; /* unused: gf_mul short-circuits zero operands */
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b)
            g_mul[a][b] = (a && b) ? g_exp[g_log[a] + g_log[b]] : 0;
    g_ready = 1;
}

/* ec_base.c:36-48 gf_mul */
uint8_t orc_gf_mul(uint8_t a, uint8_t b)
{
    orc_init();
    return g_mul[a][b];
}

/* ec_base.c:50-60 gf_inv (gf_inv(0) == 0 there as well) */
uint8_t orc_gf_inv(uint8_t a)
{
    orc_init();
    if (a == 0)
        return 0;
    return g_exp[255 - g_log[a]];
}

uint8_t orc_gf_exp(int i)
{
    orc_init();
    i %= 255;
    if (i < 0)
        i += 255;
    return g_exp[i];
}

/* ec_base.c:62-79 gf_gen_rs_matrix: identity on top, parity row p (0-based)
 * holds gen^j with gen = 2^p, i.e. a[k+p][j] = 2^(p*j). */
void orc_gen_rs_matrix(uint8_t *a, int m, int k)
{
    orc_init();
    memset(a, 0, (size_t)k * m);
    for (int i = 0; i < k; ++i)
        a[k * i + i] = 1;
    uint8_t gen = 1;
    for (int i = k; i < m; ++i) {
        uint8_t p = 1;
        for (int j = 0; j < k; ++j) {
            a[k * i + j] = p;
            p = g_mul[p][gen];
        }
        gen = g_mul[gen][2];
    }
}

/* ec_base.c:81-97 gf_gen_cauchy1_matrix: a[i][j] = 1/(i ^ j) below identity */
void orc_gen_cauchy1_matrix(uint8_t *a, int m, int k)
{
    orc_init();
    memset(a, 0, (size_t)k * m);
    for (int i = 0; i < k; ++i)
        a[k * i + i] = 1;
    uint8_t *p = &a[k * k];
    for (int i = k; i < m; ++i)
        for (int j = 0; j < k; ++j)
            *p++ = orc_gf_inv((uint8_t)(i ^ j));
}

/* ec_base.c:99-152 gf_invert_matrix: Gauss-Jordan with row swap on a zero
 * pivot; destroys `in`; returns 0, or -1 when singular. */
int orc_invert_matrix(uint8_t *in, uint8_t *out, int n)
{
    orc_init();
    memset(out, 0, (size_t)n * n);
    for (int i = 0; i < n; ++i)
        out[i * n + i] = 1;

    for (int i = 0; i < n; ++i) {
        if (in[i * n + i] == 0) {
            int j;
            for (j = i + 1; j < n; ++j)
                if (in[j * n + i])
                    break;
            if (j == n)
                return -1;
            for (int c = 0; c < n; ++c) {
                uint8_t t = in[i * n + c];
                in[i * n + c] = in[j * n + c];
                in[j * n + c] = t;
                t = out[i * n + c];
                out[i * n + c] = out[j * n + c];
                out[j * n + c] = t;
            }
        }
        uint8_t piv = orc_gf_inv(in[i * n + i]);
        for (int c = 0; c < n; ++c) {
            in[i * n + c] = g_mul[in[i * n + c]][piv];
            out[i * n + c] = g_mul[out[i * n + c]][piv];
        }
        for (int r = 0; r < n; ++r) {
            if (r == i)
                continue;
            uint8_t f = in[r * n + i];
            if (!f)
                continue;
            const uint8_t *mrow = g_mul[f];
            for (int c = 0; c < n; ++c) {
                out[r * n + c] ^= mrow[out[i * n + c]];
                in[r * n + c] ^= mrow[in[i * n + c]];
            }
        }
    }
    return 0;
}

/* ec_base.c:157-262 gf_vect_mul_init: 32-byte nibble table,
 * tbl[x] = c*x (x<16), tbl[16+x] = c*(x<<4). */
void orc_vect_mul_init(uint8_t c, uint8_t *tbl)
{
    orc_init();
    for (int x = 0; x < 16; ++x) {
        tbl[x] = g_mul[c][x];
        tbl[16 + x] = g_mul[c][x << 4];
    }
}

/* ec_highlevel_func.c:33-43 ec_init_tables */
void orc_init_tables(int k, int rows, const uint8_t *a, uint8_t *gftbls)
{
    for (int i = 0; i < rows; ++i)
        for (int j = 0; j < k; ++j) {
            orc_vect_mul_init(*a++, gftbls);
            gftbls += 32;
        }
}

/* ec_base.c:290-305 ec_encode_data_base: dest[l][i] = XOR_j src[j][i] * v_lj,
 * coefficient read back from the table as tbl[1]. */
void orc_encode_data(int len, int srcs, int dests, const uint8_t *v,
                     uint8_t *const *src, uint8_t *const *dest)
{
    orc_init();
    for (int l = 0; l < dests; ++l) {
        uint8_t *d = dest[l];
        memset(d, 0, (size_t)len);
        for (int j = 0; j < srcs; ++j) {
            uint8_t c = v[j * 32 + l * srcs * 32 + 1];
            if (!c)
                continue;
            const uint8_t *mrow = g_mul[c];
            const uint8_t *s = src[j];
            for (int i = 0; i < len; ++i)
                d[i] ^= mrow[s[i]];
        }
    }
}

/* ec_base.c:307-321 ec_encode_data_update_base: dest[l] ^= src * v[vec_i] */
void orc_encode_data_update(int len, int k, int rows, int vec_i, const uint8_t *v,
                            const uint8_t *data, uint8_t *const *dest)
{
    orc_init();
    for (int l = 0; l < rows; ++l) {
        uint8_t c = v[vec_i * 32 + l * k * 32 + 1];
        const uint8_t *mrow = g_mul[c];
        for (int i = 0; i < len; ++i)
            dest[l][i] ^= mrow[data[i]];
    }
}

/* ec_base.c:323-329 gf_vect_mul_base: dest = c * src, c = a[1] */
void orc_vect_mul(int len, const uint8_t *a, const uint8_t *src, uint8_t *dest)
{
    orc_init();
    const uint8_t *mrow = g_mul[a[1]];
    for (int i = 0; i < len; ++i)
        dest[i] = mrow[src[i]];
}

/* ------------------------------------------------------------------------ */
/* Block-level helpers mirroring benchmark/isa_throughput/isa.cpp            */
/* ------------------------------------------------------------------------ */

/* isa.cpp:69-79 isa_encoder::encode_all for one block:
 * gf_gen_rs_matrix(a, m, k); ec_init_tables(k, m-k, &a[k*k], g); encode. */
void orc_encode_block(int k, int e, int len, uint8_t *const *data, uint8_t *const *parity)
{
    int m = k + e;
    uint8_t *a = (uint8_t *)malloc((size_t)m * k);
    uint8_t *g = (uint8_t *)malloc((size_t)32 * k * (e ? e : 1));
    orc_gen_rs_matrix(a, m, k);
    orc_init_tables(k, e, &a[k * k], g);
    orc_encode_data(len, k, e, g, data, parity);
    free(a);
    free(g);
}

/* isa.cpp:169-213 isa_decoder::decode_all for one block.
 *   err_list: the `e` erased ORIGINAL indices in ascending order (std::set
 *             iteration order, isa.cpp:150-153).
 *   data:     the encoder's k source buffers (erased ones are not read),
 *   parity:   the encoder's e parity buffers,
 *   out:      e recovered buffers, out[i] <- symbol err_list[i].
 * Returns 0, or -1 for a singular decode matrix ("BAD MATRIX", :185-190).
 * The survivor order is ascending row index over the m encode rows,
 * skipping erased rows (isa.cpp:177-182, :193-197). */
int orc_decode_block(int k, int e, int len, const uint8_t *err_list,
                     uint8_t *const *data, uint8_t *const *parity, uint8_t *const *out)
{
    int m = k + e;
    uint8_t *a = (uint8_t *)malloc((size_t)m * k);
    uint8_t *b = (uint8_t *)malloc((size_t)k * k);
    uint8_t *d = (uint8_t *)malloc((size_t)k * k);
    uint8_t *c = (uint8_t *)malloc((size_t)k * (e ? e : 1));
    uint8_t *g = (uint8_t *)malloc((size_t)32 * k * (e ? e : 1));
    uint8_t *in_err = (uint8_t *)calloc((size_t)m, 1);
    uint8_t **surv = (uint8_t **)malloc(sizeof(uint8_t *) * (size_t)k);
    int rc = 0;

    orc_gen_rs_matrix(a, m, k);
    for (int i = 0; i < e; ++i)
        in_err[err_list[i]] = 1;

    for (int i = 0, r = 0; i < k; ++i, ++r) {
        while (in_err[r])
            ++r;
        memcpy(&b[k * i], &a[k * r], (size_t)k);
        surv[i] = (r < k) ? data[r] : parity[r - k];
    }
    if (orc_invert_matrix(b, d, k) < 0) {
        rc = -1;
        goto done;
    }
    for (int i = 0; i < e; ++i)
        memcpy(&c[k * i], &d[k * err_list[i]], (size_t)k);
    orc_init_tables(k, e, c, g);
    orc_encode_data(len, k, e, g, surv, out);
done:
    free(a); free(b); free(d); free(c); free(g); free(in_err); free(surv);
    return rc;
}

/* Decode coefficient rows (e x k) for an erasure list, as decode_all builds
 * them before ec_init_tables (isa.cpp:177-204).  Returns 0 / -1. */
int orc_decode_matrix(int k, int e, const uint8_t *err_list, uint8_t *c_out)
{
    int m = k + e;
    uint8_t *a = (uint8_t *)malloc((size_t)m * k);
    uint8_t *b = (uint8_t *)malloc((size_t)k * k);
    uint8_t *d = (uint8_t *)malloc((size_t)k * k);
    uint8_t *in_err = (uint8_t *)calloc((size_t)m, 1);
    int rc = 0;
    orc_gen_rs_matrix(a, m, k);
    for (int i = 0; i < e; ++i)
        in_err[err_list[i]] = 1;
    for (int i = 0, r = 0; i < k; ++i, ++r) {
        while (in_err[r])
            ++r;
        memcpy(&b[k * i], &a[k * r], (size_t)k);
    }
    if (orc_invert_matrix(b, d, k) < 0)
        rc = -1;
    else
        for (int i = 0; i < e; ++i)
            memcpy(&c_out[k * i], &d[k * err_list[i]], (size_t)k);
    free(a); free(b); free(d); free(in_err);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* Synthetic data and erasure patterns (shared definition with the engine:  */
/* storage-benchmarks_amd/csrc/rs_synth.h).  The reference fills sources    */
/* with libc rand() after srand(time(0)) (isa.cpp:56-58, :324); a seeded    */
/* counter-based generator replaces it so GPU and CPU agree byte for byte.  */
/* ------------------------------------------------------------------------ */

static inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t orc_synth_word(uint64_t seed, uint64_t row, uint64_t word)
{
    return mix64(seed * 0x9E3779B97F4A7C15ull + row * 0xD1B54A32D192ED03ull + word);
}

/* bytes [0, len) of synthetic row `row` (8 bytes per 64-bit word, LE) */
void orc_synth_row(uint64_t seed, uint64_t row, uint8_t *dst, size_t len)
{
    for (size_t w = 0; w * 8 < len; ++w) {
        uint64_t v = orc_synth_word(seed, row, w);
        for (int b = 0; b < 8 && w * 8 + b < len; ++b)
            dst[w * 8 + b] = (uint8_t)(v >> (8 * b));
    }
}

/* Erasure pattern of block `blk`: draw (r % k) until e distinct originals are
 * chosen, then list them ascending -- the isa_decoder ctor's procedure
 * (isa.cpp:137-153) driven by mix64 instead of rand(). */
void orc_erasure_pattern(uint64_t seed, uint64_t blk, int k, int e, uint8_t *err_list)
{
    uint8_t in[256];
    memset(in, 0, sizeof(in));
    if (e > k || k > 256 || e < 0)
        return;
    int have = 0;
    uint64_t ctr = 0;
    while (have < e) {
        uint64_t r = mix64(seed ^ 0xA5A5A5A55A5A5A5Aull) ^ mix64(blk * 0x2545F4914F6CDD1Dull + ctr++);
        int s = (int)(mix64(r) % (uint64_t)k);
        if (in[s])
            continue;
        in[s] = 1;
        ++have;
    }
    for (int i = 0, n = 0; i < k; ++i)
        if (in[i])
            err_list[n++] = (uint8_t)i;
}

/* erasure_code/erasure_code_base_test.c:133-213 gf_gen_decode_matrix:
 * survivors = the first k rows of the m-row code not listed in err_list
 * (ascending; decode_index), their k x k matrix inverted; when it is
 * singular and fewer than m - k rows are erased, the last survivor steps
 * `incr` rows further (incr cumulative, skipping listed parity rows in
 * err_list[nsrcerrs .. nerrs - nsrcerrs) as the loop there is bounded) until
 * an invertible set is found or the rows run out.  Decode rows: row
 * err_list[i] of the inverse for data erasures, encode row x inverse for
 * parity erasures.  err_list must be ascending (data erasures first, as
 * gen_err_list builds it).  Returns 0, or -2 (NO_INVERT_MATRIX, "BAD
 * MATRIX").  decode_index: k entries, decode_matrix: nerrs x k. */
int orc_gen_decode_matrix(const uint8_t *encode_matrix, int k, int m, const uint8_t *err_list,
                          int nerrs, uint8_t *decode_matrix, int *decode_index)
{
    orc_init();
    uint8_t *in_err = calloc((size_t)m + 1, 1);
    uint8_t *b = malloc((size_t)k * k), *inv = malloc((size_t)k * k);
    int nsrcerrs = 0, rc = 0;
    for (int i = 0; i < nerrs; ++i) {
        in_err[err_list[i]] = 1;
        nsrcerrs += err_list[i] < k;
    }
    for (int i = 0, r = 0; i < k; ++i, ++r) {
        while (in_err[r])
            ++r;
        decode_index[i] = r;
    }
    int incr = 0;
    for (;;) {
        for (int i = 0; i < k; ++i)
            memcpy(b + (size_t)k * i, encode_matrix + (size_t)k * decode_index[i], (size_t)k);
        if (orc_invert_matrix(b, inv, k) == 0)
            break;
        if (nerrs == m - k) {
            rc = -2;
            break;
        }
        ++incr;
        for (int i = nsrcerrs; i < nerrs - nsrcerrs; ++i)
            if (err_list[i] == decode_index[k - 1] + incr)
                ++incr;
        if (decode_index[k - 1] + incr >= m) {
            rc = -2;
            break;
        }
        decode_index[k - 1] += incr;
    }
    if (rc == 0) {
        for (int i = 0; i < nsrcerrs; ++i)
            memcpy(decode_matrix + (size_t)k * i, inv + (size_t)k * err_list[i], (size_t)k);
        for (int p = nsrcerrs; p < nerrs; ++p)
            for (int i = 0; i < k; ++i) {
                uint8_t s = 0;
                for (int j = 0; j < k; ++j)
                    s ^= g_mul[inv[j * k + i]][encode_matrix[(size_t)k * err_list[p] + j]];
                decode_matrix[(size_t)k * p + i] = s;
            }
    }
    free(in_err);
    free(b);
    free(inv);
    return rc;
}

/* The recovery of erasure_code_base_test.c:299-308: recov[i] =
 * buffs[decode_index[i]], then ec_init_tables + ec_encode_data_base with
 * the decode matrix.  rows: m row pointers (data 0..k-1, parity k..m-1);
 * out: nerrs rows.  Returns gen_decode_matrix's status. */
int orc_decode_general(const uint8_t *encode_matrix, int k, int m, int len,
                       const uint8_t *err_list, int nerrs, uint8_t *const *rows,
                       uint8_t *const *out)
{
    uint8_t *dm = malloc((size_t)k * (nerrs ? nerrs : 1));
    uint8_t *g = malloc((size_t)32 * k * (nerrs ? nerrs : 1));
    int *idx = malloc(sizeof(int) * (size_t)k);
    uint8_t **recov = malloc(sizeof(uint8_t *) * (size_t)k);
    int rc = orc_gen_decode_matrix(encode_matrix, k, m, err_list, nerrs, dm, idx);
    if (rc == 0 && nerrs > 0) {
        for (int i = 0; i < k; ++i)
            recov[i] = rows[idx[i]];
        orc_init_tables(k, nerrs, dm, g);
        orc_encode_data(len, k, nerrs, g, recov, out);
    }
    free(dm);
    free(g);
    free(idx);
    free(recov);
    return rc;
}
