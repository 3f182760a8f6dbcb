/*
 * rsgpu.h -- C ABI of the MI355X-native Reed-Solomon GF(2^8) erasure engine
 * (librsgpu.so).  Drop-in boundary for the hot path of
 * steinwurf/storage-benchmarks' benchmark/isa_throughput: the plugin calls
 * the ISA-L 2.13 C ABI (isa-l_open_src_2.13/isa/erasure_code.h) from
 * isa_encoder::encode_all (benchmark/isa_throughput/isa.cpp:69-79) and
 * isa_decoder::decode_all (isa.cpp:169-213).  Every entry point below names
 * the reference interface it replaces.
 *
 * Conventions (same as the ISA-L ABI):
 *   - plain pointers and sizes, C linkage, no exceptions, no allocation of
 *     caller data: the caller owns every buffer (host or device);
 *   - status returns: RSGPU_OK (0) or a negative RSGPU_ERR_* code; the
 *     context keeps a message for rsgpu_last_error();
 *   - work is enqueued on the context's HIP stream (hipStream_t passed as
 *     void*); nothing synchronises unless the function says so;
 *   - one context per device and host thread; distinct contexts are
 *     independent (one process or thread per GPU).
 *
 * Device data layout of the batched calls ("blocks"): row r of block b of a
 * buffer with R rows per block lives at base + (b*R + r)*pitch, pitch >= len.
 * Source rows are the k original symbols, parity rows the e = m-k coded
 * symbols (gf_gen_rs_matrix rows k..m-1), exactly as isa_encoder's m_buffs
 * (isa.cpp:46-58) but contiguous in HBM.
 */
#ifndef RSGPU_H
#define RSGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSGPU_OK 0
#define RSGPU_ERR_ARG (-1)
#define RSGPU_ERR_HIP (-2)
#define RSGPU_ERR_SINGULAR (-3)
#define RSGPU_ERR_NOMEM (-4)
#define RSGPU_ERR_UNSUPPORTED (-5)

#define RSGPU_MAX_SOURCES 250 /* TEST_SOURCES, isa.cpp:25-27 */

typedef struct rsgpu_ctx rsgpu_ctx;

/* ---- version / context -------------------------------------------------- */

/* "major.minor.patch" of the engine */
const char *rsgpu_version(void);

/* Binds the calling thread to HIP device `device` and creates a context whose
 * stream is the device's null stream until rsgpu_set_stream(). */
int rsgpu_create(int device, rsgpu_ctx **out);
int rsgpu_destroy(rsgpu_ctx *ctx);
/* Moves the context to another stream.  Work already enqueued on the old
 * stream is ordered before anything the context enqueues afterwards (the new
 * stream waits on an event recorded on the old one): the context's internal
 * scratch and staging buffers are never reused while an earlier kernel may
 * still read them. */
int rsgpu_set_stream(rsgpu_ctx *ctx, void *hip_stream);
void *rsgpu_get_stream(rsgpu_ctx *ctx);
int rsgpu_synchronize(rsgpu_ctx *ctx);
const char *rsgpu_last_error(rsgpu_ctx *ctx);

/* Per-kernel timing (instrumentation, off by default): while enabled every
 * kernel the engine enqueues is bracketed by HIP events on the stream it runs
 * on.  rsgpu_timing_read() synchronises the streams, writes up to `max`
 * (kernel name, milliseconds, blocks processed) records in launch order
 * (any output array may be NULL), returns how many, and
 * clears the log.  Names are static strings owned by the library. */
int rsgpu_timing_enable(rsgpu_ctx *ctx, int on);
int rsgpu_timing_read(rsgpu_ctx *ctx, const char **names, float *ms, size_t *blocks,
                      int max);

/* Device memory helpers for C/C++ callers without another allocator. */
int rsgpu_malloc(rsgpu_ctx *ctx, void **dptr, size_t bytes);
int rsgpu_free(rsgpu_ctx *ctx, void *dptr);
int rsgpu_memcpy_h2d(rsgpu_ctx *ctx, void *dst, const void *src, size_t bytes);
int rsgpu_memcpy_d2h(rsgpu_ctx *ctx, void *dst, const void *src, size_t bytes);

/* ---- host GF(2^8) helpers: the ISA-L C ABI, same arguments/semantics ----- */

/* erasure_code.h gf_mul / gf_inv (isa/ec_base.c:36-60) */
unsigned char rsgpu_gf_mul(unsigned char a, unsigned char b);
unsigned char rsgpu_gf_inv(unsigned char a);
/* erasure_code.h:898 gf_gen_rs_matrix (isa/ec_base.c:62-79) */
void rsgpu_gf_gen_rs_matrix(unsigned char *a, int m, int k);
/* erasure_code.h gf_gen_cauchy1_matrix (isa/ec_base.c:81-97) */
void rsgpu_gf_gen_cauchy1_matrix(unsigned char *a, int m, int k);
/* erasure_code.h:924 gf_invert_matrix (isa/ec_base.c:99-152): destroys `in`,
 * returns 0 or -1 when singular. */
int rsgpu_gf_invert_matrix(unsigned char *in, unsigned char *out, const int n);
/* erasure_code.h gf_vect_mul_init (isa/ec_base.c:157-262): 32-byte table */
void rsgpu_gf_vect_mul_init(unsigned char c, unsigned char *tbl);
/* erasure_code.h:74 ec_init_tables (isa/ec_highlevel_func.c:33-43) */
void rsgpu_ec_init_tables(int k, int rows, unsigned char *a, unsigned char *gftbls);

/* ---- device, ISA-L-shaped ------------------------------------------------ */

/* erasure_code.h:98 ec_encode_data (isa/ec_multibinary.asm:112-162 dispatch,
 * isa/ec_highlevel_func.c:106-135 avx2 split): coding[r][i] =
 * XOR_j c[r][j]*data[j][i].  `gftbls` is HOST memory in ISA-L's 32-byte table
 * format (as produced by ec_init_tables); `data` / `coding` are HOST arrays
 * of DEVICE pointers; any len >= 0 and any alignment. */
int rsgpu_ec_encode_data(rsgpu_ctx *ctx, int len, int k, int rows, const unsigned char *gftbls,
                         unsigned char **data, unsigned char **coding);

/* erasure_code.h ec_encode_data_update (isa/ec_highlevel_func.c:139-252,
 * isa/ec_base.c:307-321): coding[r][i] ^= c[r][vec_i] * data[i]. */
int rsgpu_ec_encode_data_update(rsgpu_ctx *ctx, int len, int k, int rows, int vec_i,
                                const unsigned char *gftbls, unsigned char *data,
                                unsigned char **coding);

/* The single-output / single-source members of the same ABI, as
 * isa_arithmetic and ISA-L's own tests call them (HOST tables and pointer
 * arrays, DEVICE rows, as rsgpu_ec_encode_data):
 *   erasure_code.h:637 gf_vect_dot_prod (isa/ec_base.c:264-276
 *     gf_vect_dot_prod_base): dest[i] = XOR_j c[j] * src[j][i], the 32*vlen
 *     tables of ONE output row; any len >= 0 (ISA-L asks len >= 32).
 *   erasure_code.h:664 gf_vect_mad (isa/ec_base.c:278-288): dest[i] ^=
 *     c[vec_i] * src[i], tables of vec coefficients.
 *   gf_vect_mul.h:108 gf_vect_mul (isa/ec_base.c:323-329): dest[i] =
 *     c * src[i] with c = gftbl[1]; returns 0, or non-zero when len is not a
 *     multiple of 32 (the dispatched ISA-L function's contract). */
int rsgpu_gf_vect_dot_prod(rsgpu_ctx *ctx, int len, int vlen, const unsigned char *gftbls,
                           unsigned char **src, unsigned char *dest);
int rsgpu_gf_vect_mad(rsgpu_ctx *ctx, int len, int vec, int vec_i, const unsigned char *gftbls,
                      unsigned char *src, unsigned char *dest);
int rsgpu_gf_vect_mul(rsgpu_ctx *ctx, int len, const unsigned char *gftbl, void *src, void *dest);

/* ---- device, batched blocks (the benchmark hot path) --------------------- */

/* isa_encoder::encode_all over `blocks` independent blocks (isa.cpp:69-79):
 * parity[b][p] = XOR_j a[k+p][j] * src[b][j] with a = gf_gen_rs_matrix(k+e, k)
 * when `coef` is NULL, else with the HOST e x k row-major matrix `coef`.
 * src: [blocks][k] rows, parity: [blocks][e] rows, both at `pitch`. */
int rsgpu_encode_blocks(rsgpu_ctx *ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                        const unsigned char *d_src, unsigned char *d_parity,
                        const unsigned char *coef);

/* Encode kernel of rsgpu_encode_blocks / rsgpu_ec_encode_data (per context;
 * every choice writes the same bytes):
 *   AUTO       COMPILED for the codes built in (gf_gen_rs_matrix (k, e) in
 *              {(16,4) (16,8) (64,32) (64,16) (5,4) (20,7)}, no `coef`),
 *              otherwise GENERATED (aligned rows, len % 32 == 0; (100,20),
 *              compiled too, runs GENERATED: its compiled waves own 5 rows),
 *              otherwise the v_perm kernel
 *   COMPILED   k_rs_bs: the matrix compiled into the kernel (codes above
 *              and (100,20))
 *   GENERATED  code built on the host for the matrix, once, shared by every
 *              block: per (wave, source) only the composites its
 *              coefficients need (greedy cover); 2 waves x 16 / 12 / 10 rows
 *              for 16 < e <= 32, 4 waves for 32 < e <= 64, passes of <= 64
 *              rows above (k_rs_jitw, the decode's layout), else waves of 8
 *              rows (k_rs_jit); the context keeps the last 64 programs (at
 *              most 256 MB of executable device memory, least recently
 *              used out), so a caller cycling through matrices builds each
 *              once
 *   THREADED   k_rs_tc: 256 generated handlers, one dispatch per coefficient
 * A choice that does not apply falls back in that order. */
#define RSGPU_ENCODE_AUTO 0
#define RSGPU_ENCODE_COMPILED 1
#define RSGPU_ENCODE_GENERATED 2
#define RSGPU_ENCODE_THREADED 3
int rsgpu_set_encode_kernel(rsgpu_ctx *ctx, int kernel);

/* Device workspace needed by rsgpu_decode_blocks for this geometry (any
 * decode kernel choice). */
size_t rsgpu_decode_workspace_bytes(int k, int e, size_t blocks);

/* Decode kernel of rsgpu_decode_blocks (per context; every choice recovers
 * the same bytes):
 *   AUTO        GENERATED when a block has >= 16 column tiles of 2 KB
 *               (len > 30 KiB), or fewer whose generated code is at most
 *               2 KB per tile, and the call has >= 4096 (block, tile)
 *               pairs, else ONE_MATRIX (the default)
 *   ONE_MATRIX  closed-form e x k decode rows V_E^-1 [V_kept | I] (e <= 32),
 *               one threaded-code pass over the k - e survivors + e parity;
 *               rsgpu_decode_blocks runs a small call (< 2048 (block, 2 KB
 *               column) pairs, e <= 8, k <= 64) as ONE launch that builds the
 *               rows itself (the prepare/apply pair keeps two); under AUTO a
 *               small call of a code with a compiled single-chunk program
 *               ((16,4) (16,8) (5,4) (20,7)) instead runs ONE launch of
 *               syndromes through that program plus the e x e solve
 *   GENERAL     the reference's k x k survivor-matrix inversion on the
 *               device (isa.cpp:177-204), then the decode rows; any e
 *   GENERATED   the ONE_MATRIX rows baked into per-block straight-line code
 *               (written to executable device memory by the prepare step),
 *               one call per chunk of sources: 2 waves x 16 rows for
 *               24 < e <= 32 (k_rs_jit16), x 12 rows for 20 < e <= 24
 *               (k_rs_jit12), x 10 rows for 16 < e <= 20 (k_rs_jit10),
 *               4 waves of 10 / 12 / 16 rows for 32 < e <= 40 / 48 / 64
 *               (k_rs_jit{10,12,16}x4), passes of <= 64 rows for e > 64
 *               (closed-form rows for every e; AUTO takes it for e > 32
 *               when the code pays for itself -- enough column tiles per
 *               block, jit_pays -- and otherwise runs GENERAL), else waves
 *               of 8 rows (k_rs_jit, e <= 16)
 * A choice that does not apply to a geometry falls back to GENERAL (e > 32,
 * unaligned rows) or ONE_MATRIX. */
#define RSGPU_DECODE_AUTO 0
#define RSGPU_DECODE_ONE_MATRIX 1
/* Deprecated alias: 2 selected a fused syndrome + solve kernel (removed in
 * round 3, never faster).  It is still accepted and runs ONE_MATRIX, which
 * writes the same bytes. */
#define RSGPU_DECODE_FUSED 2
#define RSGPU_DECODE_GENERAL 3
#define RSGPU_DECODE_GENERATED 4
int rsgpu_set_decode_kernel(rsgpu_ctx *ctx, int kernel);

/* isa_decoder::decode_all over `blocks` blocks (isa.cpp:169-213): for block
 * b the `e` erased ORIGINAL indices d_err[b][0..e-1] (strictly ascending, as
 * the std::set iterates, isa.cpp:150-153) are rebuilt from the surviving
 * originals and all e parity rows.  On the device: survivor matrix ->
 * gf_invert_matrix -> decode rows -> dot product into out[b][i] (symbol
 * d_err[b][i]).  The erased rows of d_src are never read.  d_status[b] = 0;
 * -1 for a singular matrix ("BAD MATRIX", isa.cpp:185-190); -2 for a
 * malformed erasure list (not strictly ascending, or an index >= k).  A
 * block with a non-zero status is skipped; its output is unspecified.
 * d_workspace holds rsgpu_decode_workspace_bytes() bytes.  Batches of more
 * than 65535 blocks run as consecutive slices (as do rsgpu_encode_blocks,
 * rsgpu_decode_general and rsgpu_verify_blocks). */
int rsgpu_decode_blocks(rsgpu_ctx *ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                        const unsigned char *d_src, const unsigned char *d_parity,
                        const unsigned char *d_err, unsigned char *d_out, void *d_workspace,
                        int *d_status);

/* The two halves of rsgpu_decode_blocks, for callers that time or reuse them:
 * prepare = survivor matrix + gf_invert_matrix + decode tables + row pointers
 * (isa.cpp:177-207) into d_workspace and d_status; apply = the dot product
 * (isa.cpp:208-209) for blocks whose status is 0.  decode_blocks ==
 * prepare followed by apply on the same stream.  At most 65535 blocks per
 * call (RSGPU_ERR_ARG beyond).  apply must be given the geometry, block
 * count, buffers and workspace of the prepare before it, with no
 * rsgpu_set_decode_kernel in between: both derive the decode kernel (and so
 * the workspace layout) from them.  The generated-code decode keeps the code
 * of the context's LAST prepare: an apply whose (k, e, blocks, workspace)
 * differ from it, or that follows another decode call on the context (which
 * rewrites or regrows the code), returns RSGPU_ERR_ARG and launches nothing. */
int rsgpu_decode_prepare(rsgpu_ctx *ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                         const unsigned char *d_src, const unsigned char *d_parity,
                         const unsigned char *d_err, unsigned char *d_out, void *d_workspace,
                         int *d_status);
int rsgpu_decode_apply(rsgpu_ctx *ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                       const unsigned char *d_src, const unsigned char *d_parity,
                       unsigned char *d_out, void *d_workspace, const int *d_status);

/* General erasure decode: ISA-L's gf_gen_decode_matrix + recovery
 * (isa-l_open_src_2.13/erasure_code/erasure_code_base_test.c:133-213, :292-
 * 308) for any m x k encode matrix and erasures among data AND parity rows.
 *   encode_matrix  HOST m x k row-major (identity on top, as gf_gen_rs_matrix
 *                  / gf_gen_cauchy1_matrix make it), or NULL for
 *                  gf_gen_rs_matrix(m, k)
 *   d_src [blocks][k] rows, d_parity [blocks][m-k] rows (pitch `pitch`)
 *   d_err [blocks][nerrs] erased row indices in [0, m), strictly ascending
 *   d_out [blocks][nerrs] recovered rows, in d_err order
 * Survivors are the first k rows not erased, ascending; when their matrix is
 * singular the reference's retry (replace the last survivor by a later row,
 * :163-184) runs, and only when that fails the block gets status -1 ("BAD
 * MATRIX").  Status -2: malformed list (not ascending, index >= m, or more
 * than m - k erasures).  Erased rows are never read. */
size_t rsgpu_decode_general_workspace_bytes(int k, int m, int nerrs, size_t blocks);
int rsgpu_decode_general(rsgpu_ctx *ctx, int k, int m, size_t len, size_t pitch, size_t blocks,
                         const unsigned char *encode_matrix, const unsigned char *d_src,
                         const unsigned char *d_parity, const unsigned char *d_err, int nerrs,
                         unsigned char *d_out, void *d_workspace, int *d_status);

/* isa_decoder::verify_data (isa.cpp:215-229) on the device: adds to
 * d_mismatch[b] the number of bytes where out[b][i] != src[b][d_err[b][i]]. */
int rsgpu_verify_blocks(rsgpu_ctx *ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                        const unsigned char *d_src, const unsigned char *d_out,
                        const unsigned char *d_err, unsigned long long *d_mismatch);

/* ---- host-resident blocks (the reference's buffers, isa.cpp:46-58) ------- */

/* Page-locked host memory for the host-resident calls: their copies then run
 * as DMA at the link rate and overlap the kernels (pageable memory works,
 * but is copied synchronously, so the stages run in series). */
int rsgpu_host_alloc(rsgpu_ctx *ctx, void **hptr, size_t bytes);
int rsgpu_host_free(rsgpu_ctx *ctx, void *hptr);

/* isa_encoder::encode_all over blocks held in HOST memory, as isa.cpp:46-58
 * holds them (isa.cpp:69-79): h_src [blocks][k] rows, h_parity [blocks][e]
 * rows, at `pitch` >= len.  The batch streams through device staging in
 * chunks, copy-in / rsgpu_encode_blocks / copy-out of consecutive chunks
 * overlapped on three streams.  Synchronous: the parity is in h_parity on
 * return.  `coef` as rsgpu_encode_blocks. */
int rsgpu_encode_blocks_host(rsgpu_ctx *ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                             const unsigned char *h_src, unsigned char *h_parity,
                             const unsigned char *coef);

/* isa_decoder::decode_all over HOST-resident blocks (isa.cpp:169-213): the
 * erasure lists h_err [blocks][e] as rsgpu_decode_blocks; only what the
 * reference's decoder reads crosses the link towards the GPU -- the surviving
 * originals (as runs of consecutive rows; rows shorter than 64 KiB go as
 * whole blocks, erased rows included, which the kernels never read) and the
 * parity rows -- and the recovered rows land in h_out [blocks][e] (in h_err
 * order).  h_status [blocks] (may be NULL) receives rsgpu_decode_blocks'
 * per-block status.  Pipelined and synchronous as rsgpu_encode_blocks_host. */
int rsgpu_decode_blocks_host(rsgpu_ctx *ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                             const unsigned char *h_src, const unsigned char *h_parity,
                             const unsigned char *h_err, unsigned char *h_out, int *h_status);

/* ---- synthetic workload (replaces rand(), isa.cpp:56-58, :137-146) ------- */

/* Fills `rows` rows of `len` bytes at `pitch` with the seeded counter-based
 * stream: bytes 8w..8w+7 of global row (row0 + r) = LE(mix(seed, row, w)). */
int rsgpu_fill_synthetic(rsgpu_ctx *ctx, unsigned char *d_rows, size_t rows, size_t len,
                         size_t pitch, uint64_t seed, uint64_t row0);

/* Host: erasure lists of blocks blk0..blk0+blocks-1 into h_err[blocks][e]
 * (e distinct originals per block, ascending), as the isa_decoder ctor draws
 * them (isa.cpp:137-153) with a seeded generator. */
int rsgpu_erasure_patterns(uint64_t seed, uint64_t blk0, size_t blocks, int k, int e,
                           unsigned char *h_err);

#ifdef __cplusplus
}
#endif

#endif /* RSGPU_H */
