/*
 * ref_driver.c -- thin driver around the UNMODIFIED ISA-L 2.13 base C
 * (isa/ec_base.c, isa/ec_highlevel_func.c) compiled straight from
 * /root/reference by oracle/Makefile into oracle/_ref/libisal_ref.so
 * (TEST INFRASTRUCTURE ONLY -- the engine never links it).
 *
 * The driver plays the role benchmark/isa_throughput/isa.cpp plays in the
 * reference: it calls gf_gen_rs_matrix / ec_init_tables / ec_encode_data_base /
 * gf_invert_matrix exactly as isa_encoder::encode_all (isa.cpp:69-79) and
 * isa_decoder::decode_all (isa.cpp:169-213) do.  The AVX2 assembly kernels
 * cannot be assembled in this image (no yasm/nasm), so the
 * dispatched ec_encode_data is replaced by the reference's own scalar
 * ec_encode_data_base, which ISA-L's tests pin as bit-identical to the asm
 * (erasure_code/gf_vect_dot_prod_avx_test.c:162-193).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#include "erasure_code.h"

/* ec_base.c functions that erasure_code.h does not declare in 2.13 */
void ec_encode_data_base(int len, int srcs, int dests, unsigned char *v,
                         unsigned char **src, unsigned char **dest);
void ec_encode_data_update_base(int len, int k, int rows, int vec_i, unsigned char *v,
                                unsigned char *data, unsigned char **dest);
void gf_vect_mul_base(int len, unsigned char *a, unsigned char *src, unsigned char *dest);

unsigned char ref_gf_mul(unsigned char a, unsigned char b) { return gf_mul(a, b); }
unsigned char ref_gf_inv(unsigned char a) { return gf_inv(a); }
void ref_gf_gen_rs_matrix(unsigned char *a, int m, int k) { gf_gen_rs_matrix(a, m, k); }
void ref_gf_gen_cauchy1_matrix(unsigned char *a, int m, int k) { gf_gen_cauchy1_matrix(a, m, k); }
int ref_gf_invert_matrix(unsigned char *in, unsigned char *out, int n)
{
    return gf_invert_matrix(in, out, n);
}
void ref_gf_vect_mul_init(unsigned char c, unsigned char *tbl) { gf_vect_mul_init(c, tbl); }
void ref_ec_init_tables(int k, int rows, unsigned char *a, unsigned char *g)
{
    ec_init_tables(k, rows, a, g);
}
void ref_ec_encode_data(int len, int k, int rows, unsigned char *g, unsigned char **data,
                        unsigned char **coding)
{
    ec_encode_data_base(len, k, rows, g, data, coding);
}
void ref_ec_encode_data_update(int len, int k, int rows, int vec_i, unsigned char *g,
                               unsigned char *data, unsigned char **coding)
{
    ec_encode_data_update_base(len, k, rows, vec_i, g, data, coding);
}
void ref_gf_vect_mul(int len, unsigned char *a, unsigned char *src, unsigned char *dest)
{
    gf_vect_mul_base(len, a, src, dest);
}

/* The data kernel of the timed regions: the reference's scalar
 * ec_encode_data_base, or the AVX2 restatement of its asm path
 * (isal_avx2_port.c; CPU baseline only). */
typedef void (*data_kernel_t)(int, int, int, unsigned char *, unsigned char **, unsigned char **);
void port_ec_encode_data_avx2(int len, int k, int rows, unsigned char *g, unsigned char **data,
                              unsigned char **coding);
int port_have_avx2(void);

static void encode_block_with(data_kernel_t kern, int k, int e, int len, unsigned char **data,
                              unsigned char **parity);
static int decode_block_with(data_kernel_t kern, int k, int e, int len,
                             const unsigned char *err_list, unsigned char **data,
                             unsigned char **parity, unsigned char **out);

/* isa.cpp:69-79 */
void ref_encode_block(int k, int e, int len, unsigned char **data, unsigned char **parity)
{
    encode_block_with(ec_encode_data_base, k, e, len, data, parity);
}

/* isa.cpp:169-213 (err_list ascending, as std::set iterates) */
int ref_decode_block(int k, int e, int len, const unsigned char *err_list,
                     unsigned char **data, unsigned char **parity, unsigned char **out)
{
    return decode_block_with(ec_encode_data_base, k, e, len, err_list, data, parity, out);
}

/* the AVX2 port through the same flow (tests pin it against the base C) */
void ref_encode_block_avx2(int k, int e, int len, unsigned char **data, unsigned char **parity)
{
    encode_block_with(port_ec_encode_data_avx2, k, e, len, data, parity);
}

int ref_decode_block_avx2(int k, int e, int len, const unsigned char *err_list,
                          unsigned char **data, unsigned char **parity, unsigned char **out)
{
    return decode_block_with(port_ec_encode_data_avx2, k, e, len, err_list, data, parity, out);
}

int ref_have_avx2(void) { return port_have_avx2(); }

static void encode_block_with(data_kernel_t kern, int k, int e, int len, unsigned char **data,
                              unsigned char **parity)
{
    int m = k + e;
    unsigned char *a = malloc((size_t)m * k);
    unsigned char *g = malloc((size_t)32 * k * (e ? e : 1));
    gf_gen_rs_matrix(a, m, k);
    ec_init_tables(k, m - k, &a[k * k], g);
    kern(len, k, m - k, g, data, parity);
    free(a);
    free(g);
}

static int decode_block_with(data_kernel_t kern, int k, int e, int len,
                             const unsigned char *err_list, unsigned char **data,
                             unsigned char **parity, unsigned char **out)
{
    int m = k + e, rc = 0;
    unsigned char *a = malloc((size_t)m * k), *b = malloc((size_t)k * k);
    unsigned char *d = malloc((size_t)k * k), *c = malloc((size_t)k * (e ? e : 1));
    unsigned char *g = malloc((size_t)32 * k * (e ? e : 1));
    unsigned char *in_err = calloc((size_t)m, 1);
    unsigned char **surv = malloc(sizeof(unsigned char *) * (size_t)k);
    gf_gen_rs_matrix(a, m, k);
    for (int i = 0; i < e; ++i)
        in_err[err_list[i]] = 1;
    for (int i = 0, r = 0; i < k; ++i, ++r) {
        while (in_err[r])
            ++r;
        for (int j = 0; j < k; ++j)
            b[k * i + j] = a[k * r + j];
        surv[i] = r < k ? data[r] : parity[r - k];
    }
    if (gf_invert_matrix(b, d, k) < 0) {
        rc = -1;
    } else {
        for (int i = 0; i < e; ++i)
            for (int j = 0; j < k; ++j)
                c[k * i + j] = d[k * err_list[i] + j];
        ec_init_tables(k, e, c, g);
        kern(len, k, e, g, surv, out);
    }
    free(a); free(b); free(d); free(c); free(g); free(in_err); free(surv);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* CPU baseline: isa_throughput's timed regions (encode = matrix + tables +  */
/* kernel; decode = inversion + tables + kernel) over independent blocks,    */
/* one block per thread at a time.  Inputs are generated outside the timed   */
/* region, as the reference's constructors do (throughput_benchmark.hpp:     */
/* 165-177).                                                                 */
/* ------------------------------------------------------------------------ */

/* Row buffers of the CPU baseline: each its own anonymous mapping, so every
 * row starts on a page boundary whatever the allocator did before.  (With
 * glibc's aligned_alloc the rows came from mmap on a fresh process but from
 * the heap after earlier frees had raised the mmap threshold; in that state
 * the port's decode ran at 1.5-2x its encode time on the GPU box's host,
 * tools/cpu_asym.py, profiles/r02_cpu_asym.json.) */
static unsigned char *row_alloc(size_t len)
{
    void *p = mmap(NULL, len ? len : 1, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    return p == MAP_FAILED ? NULL : (unsigned char *)p;
}

static void row_free(unsigned char *p, size_t len)
{
    if (p)
        munmap(p, len ? len : 1);
}

static inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

typedef struct {
    int k, e, len, blocks_per_thread, tid;
    data_kernel_t kern;
    uint64_t seed;
    double enc_s, dec_s;
    int failures;
} job_t;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *worker(void *arg)
{
    job_t *j = (job_t *)arg;
    int k = j->k, e = j->e, len = j->len, m = k + e;
    unsigned char **data = malloc(sizeof(void *) * (size_t)k);
    unsigned char **par = malloc(sizeof(void *) * (size_t)(e ? e : 1));
    unsigned char **out = malloc(sizeof(void *) * (size_t)(e ? e : 1));
    for (int i = 0; i < k; ++i)
        data[i] = row_alloc((size_t)len);
    for (int i = 0; i < e; ++i) {
        par[i] = row_alloc((size_t)len);
        out[i] = row_alloc((size_t)len);
    }
    /* outputs pre-touched outside the timed region, so the timed kernels do
     * not pay first-touch page faults (the reference's posix_memalign'd
     * parity buffers would; this favours the CPU baseline) */
    for (int i = 0; i < e; ++i) {
        memset(par[i], 0, (size_t)len);
        memset(out[i], 0, (size_t)len);
    }
    unsigned char err[256], in_err[256];
    /* for the AVX2 port, block -1 warms the thread up (first touch of the
     * allocator's and the kernel's working memory; a 1-thread sample's first
     * encode measured up to 2.5x the next) and is not counted; the scalar
     * reference kernel is slow enough not to need it */
    const int first = j->kern == port_ec_encode_data_avx2 ? -1 : 0;
    for (int b = first; b < j->blocks_per_thread; ++b) {
        uint64_t blk = (uint64_t)j->tid * 1000003ull + (uint64_t)(b + 1);
        for (int i = 0; i < k; ++i)
            for (int p = 0; p < len; p += 8) {
                uint64_t v = mix64(j->seed * 0x9E3779B97F4A7C15ull + (blk * k + i) * 0xD1B54A32D192ED03ull + (uint64_t)p / 8);
                for (int q = 0; q < 8 && p + q < len; ++q)
                    data[i][p + q] = (unsigned char)(v >> (8 * q));
            }
        memset(in_err, 0, sizeof(in_err));
        for (int have = 0, ctr = 0; have < e; ++ctr) {
            int s = (int)(mix64(j->seed ^ (blk * 0x2545F4914F6CDD1Dull) ^ (uint64_t)ctr) % (uint64_t)k);
            if (!in_err[s]) {
                in_err[s] = 1;
                ++have;
            }
        }
        for (int i = 0, n = 0; i < k; ++i)
            if (in_err[i])
                err[n++] = (unsigned char)i;
        double t0 = now_s();
        encode_block_with(j->kern, k, e, len, data, par);
        double t1 = now_s();
        int rc = decode_block_with(j->kern, k, e, len, err, data, par, out);
        double t2 = now_s();
        if (b >= 0) {
            j->enc_s += t1 - t0;
            j->dec_s += t2 - t1;
        }
        if (rc != 0)
            j->failures++;
        else
            for (int i = 0; i < e; ++i)
                if (memcmp(out[i], data[err[i]], (size_t)len))
                    j->failures++;
    }
    for (int i = 0; i < k; ++i)
        row_free(data[i], (size_t)len);
    for (int i = 0; i < e; ++i) {
        row_free(par[i], (size_t)len);
        row_free(out[i], (size_t)len);
    }
    free(data); free(par); free(out);
    (void)m;
    return NULL;
}

/* Runs `threads` workers, each encoding+decoding `blocks_per_thread` blocks
 * with data kernel `kernel` (0 = reference ec_encode_data_base, 1 = AVX2
 * port).  Returns wall seconds of the whole run; *enc_s / *dec_s are the
 * summed per-block timed-region seconds, *max_thread_s the largest
 * per-thread sum of both; *failures counts unrecovered symbols. */
double ref_cpu_bench_kernel(int k, int e, int len, int threads, int blocks_per_thread,
                            uint64_t seed, int kernel, double *enc_s, double *dec_s,
                            double *max_thread_s, int *failures);

double ref_cpu_bench(int k, int e, int len, int threads, int blocks_per_thread, uint64_t seed,
                     double *enc_s, double *dec_s, double *max_thread_s, int *failures)
{
    return ref_cpu_bench_kernel(k, e, len, threads, blocks_per_thread, seed, 0, enc_s, dec_s,
                                max_thread_s, failures);
}

double ref_cpu_bench_kernel(int k, int e, int len, int threads, int blocks_per_thread,
                            uint64_t seed, int kernel, double *enc_s, double *dec_s,
                            double *max_thread_s, int *failures)
{
    job_t *jobs = calloc((size_t)threads, sizeof(job_t));
    pthread_t *th = calloc((size_t)threads, sizeof(pthread_t));
    double t0 = now_s();
    for (int t = 0; t < threads; ++t) {
        jobs[t].k = k; jobs[t].e = e; jobs[t].len = len;
        jobs[t].blocks_per_thread = blocks_per_thread; jobs[t].tid = t; jobs[t].seed = seed;
        jobs[t].kern = kernel == 1 ? port_ec_encode_data_avx2 : ec_encode_data_base;
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    double es = 0, ds = 0, mx = 0;
    int f = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        es += jobs[t].enc_s;
        ds += jobs[t].dec_s;
        if (jobs[t].enc_s + jobs[t].dec_s > mx)
            mx = jobs[t].enc_s + jobs[t].dec_s;
        f += jobs[t].failures;
    }
    *max_thread_s = mx;
    double wall = now_s() - t0;
    *enc_s = es;
    *dec_s = ds;
    *failures = f;
    free(jobs);
    free(th);
    return wall;
}

/* ------------------------------------------------------------------------ */
/* Diagnostic for the CPU baseline's decode/encode asymmetry (bench.py       */
/* reports the port's decode at ~2x its encode on the GPU box): one thread,  */
/* the worker's allocation and generation pattern, per rep:                  */
/*   t[0] encode_block_with (as timed by the baseline)                       */
/*   t[1] decode_block_with (as timed by the baseline)                       */
/*   t[2] the decode's data kernel alone, same survivors and outputs, again  */
/*   t[3] the encode's data kernel alone, again                              */
/*   t[4] the decode's data kernel into fresh (pre-touched) outputs          */
/* ------------------------------------------------------------------------ */
void ref_cpu_asym(int k, int e, int len, int reps, double *t)
{
    unsigned char **data = malloc(sizeof(void *) * (size_t)k);
    unsigned char **par = malloc(sizeof(void *) * (size_t)e);
    unsigned char **out = malloc(sizeof(void *) * (size_t)e);
    unsigned char **out2 = malloc(sizeof(void *) * (size_t)e);
    unsigned char **surv = malloc(sizeof(void *) * (size_t)k);
    for (int i = 0; i < k; ++i)
        data[i] = row_alloc((size_t)len);
    for (int i = 0; i < e; ++i) {
        par[i] = row_alloc((size_t)len);
        out[i] = row_alloc((size_t)len);
        out2[i] = row_alloc((size_t)len);
        memset(par[i], 0, (size_t)len);
        memset(out[i], 0, (size_t)len);
        memset(out2[i], 0, (size_t)len);
    }
    int m = k + e;
    unsigned char *a = malloc((size_t)m * k), *g = malloc((size_t)32 * k * e);
    unsigned char err[256], in_err[256];
    gf_gen_rs_matrix(a, m, k);
    ec_init_tables(k, e, &a[k * k], g);
    for (int q = 0; q < 5; ++q)
        t[q] = 0;
    for (int r = 0; r < reps; ++r) {
        for (int i = 0; i < k; ++i)
            for (int p = 0; p < len; p += 8) {
                uint64_t v = mix64((uint64_t)r * 0x9E3779B97F4A7C15ull + (uint64_t)i * 0xD1B54A32D192ED03ull + (uint64_t)p / 8);
                for (int q = 0; q < 8 && p + q < len; ++q)
                    data[i][p + q] = (unsigned char)(v >> (8 * q));
            }
        memset(in_err, 0, sizeof(in_err));
        for (int have = 0, ctr = 0; have < e; ++ctr) {
            int s = (int)(mix64((uint64_t)r * 0x2545F4914F6CDD1Dull ^ (uint64_t)ctr) % (uint64_t)k);
            if (!in_err[s]) {
                in_err[s] = 1;
                ++have;
            }
        }
        for (int i = 0, n = 0; i < k; ++i)
            if (in_err[i])
                err[n++] = (unsigned char)i;
        for (int i = 0, q = 0; i < k; ++i)
            if (!in_err[i])
                surv[q++] = data[i];
        for (int i = 0; i < e; ++i)
            surv[k - e + i] = par[i];
        double t0 = now_s();
        encode_block_with(port_ec_encode_data_avx2, k, e, len, data, par);
        double t1 = now_s();
        decode_block_with(port_ec_encode_data_avx2, k, e, len, err, data, par, out);
        double t2 = now_s();
        port_ec_encode_data_avx2(len, k, e, g, surv, out);
        double t3 = now_s();
        port_ec_encode_data_avx2(len, k, e, g, data, par);
        double t4 = now_s();
        port_ec_encode_data_avx2(len, k, e, g, surv, out2);
        double t5 = now_s();
        t[0] += t1 - t0;
        t[1] += t2 - t1;
        t[2] += t3 - t2;
        t[3] += t4 - t3;
        t[4] += t5 - t4;
    }
    for (int q = 0; q < 5; ++q)
        t[q] /= reps;
    for (int i = 0; i < k; ++i)
        row_free(data[i], (size_t)len);
    for (int i = 0; i < e; ++i) {
        row_free(par[i], (size_t)len);
        row_free(out[i], (size_t)len);
        row_free(out2[i], (size_t)len);
    }
    free(data); free(par); free(out); free(out2); free(surv); free(a); free(g);
}

typedef struct {
    int k, e, len, reps;
    double *t;
} asym_job_t;

static void *asym_worker(void *arg)
{
    asym_job_t *j = (asym_job_t *)arg;
    ref_cpu_asym(j->k, j->e, j->len, j->reps, j->t);
    return NULL;
}

/* ref_cpu_asym on a fresh pthread, as the baseline's workers run */
void ref_cpu_asym_thread(int k, int e, int len, int reps, double *t)
{
    asym_job_t j = {k, e, len, reps, t};
    pthread_t th;
    pthread_create(&th, NULL, asym_worker, &j);
    pthread_join(th, NULL);
}
