// rs_kernels.h -- launch interface of the HIP kernels (internal to librsgpu).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsgpu {

struct DotArgs {
    const uint8_t* const* srcs;   // device [blocks][k] row pointers
    uint8_t* const* dsts;         // device [blocks][rows] row pointers
    const uint4* tabs4;           // device [blocks?][k][rows_pad] (perm tables, bits 0-5)
    const uint32_t* ctab;         // device [blocks?][k][rows_pad] (perm table, bits 6-7)
    long long tab_block_stride;   // coefficients between blocks' tables (0 = shared)
    int k, rows, rows_pad;
    long long len;                // bytes per row
    long long blocks;
    const int* status;            // optional [blocks]: skip blocks with status != 0
    bool bytewise;                // pointers not 8-byte aligned: byte kernel
};

// General decode preparation (k_decode_prepare, one workgroup per block):
// survivors = the first k rows of the m-row code not erased (ascending),
// their k x k matrix inverted (Gauss-Jordan, isa/ec_base.c:99-152), with the
// reference's retry when singular (erasure_code_base_test.c:163-184); decode
// rows = inverse rows of erased data rows, encode row x inverse for erased
// parity rows (:197-210).
struct PrepArgs {
    int k, m, nerrs, rows_pad;
    long long blocks;
    const uint8_t* err;           // device [blocks][nerrs], strictly ascending, < m
    const uint8_t* enc;           // device m x k encode matrix, nullptr = gf_gen_rs_matrix(m, k)
    int originals_only;           // isa_decoder form: every erased index must be < k
    const uint8_t* src; long long src_pitch;   // [blocks][k] rows
    const uint8_t* par; long long par_pitch;   // [blocks][m - k] rows
    uint8_t* out; long long out_pitch;         // [blocks][nerrs] rows
    const uint8_t** surv_ptrs;    // device [blocks][k]
    uint8_t** out_ptrs;           // device [blocks][nerrs]
    uint4* tabs4; uint32_t* ctab; long long tab_block_stride;  // v_perm tables, or nullptr
    int* status;                  // device [blocks]
    // k_rs_tc instead of k_dot_generic (when non-null): the context's
    // 2048-entry handler table and the address output, tc_block_stride
    // elements per block in the pass layout of tc_table_elems()
    const unsigned long long* tc_table = nullptr;
    unsigned long long* tc_addr = nullptr;
    long long tc_block_stride = 0;
    // or (when non-null) the decode rows themselves, [blocks][nerrs][k], for
    // k_jit_emit
    uint8_t* coef_out = nullptr;
};

int generic_rows_per_pass(int rows);
hipError_t launch_dot_generic(const DotArgs& a, hipStream_t st);
bool rs_encode_specialized_available(int k, int e);
hipError_t launch_rs_encode_specialized(int k, int e, const uint8_t* src, uint8_t* par,
                                        long long pitch, long long len, long long blocks,
                                        hipStream_t st);
size_t decode_prepare_lds_bytes(int k);
hipError_t launch_decode_prepare(const PrepArgs& a, hipStream_t st);
hipError_t launch_fill_synth(uint8_t* dst, long long rows, long long len, long long pitch,
                             unsigned long long seed, unsigned long long row0, hipStream_t st);
hipError_t launch_compare_rows(const uint8_t* src, long long src_pitch, int k, const uint8_t* out,
                               long long out_pitch, int e, const uint8_t* err, long long len,
                               long long blocks, unsigned long long* mismatches, hipStream_t st);
// Bit-sliced RS(k, e) parity of the gf_gen_rs_matrix code with compile-time
// coefficients (rs_bitsliced.hip).  Requires len % 32 == 0, 16-byte aligned
// rows.
bool rs_bitsliced_available(int k, int e);
// output rows each wave of the compiled kernel owns (its composites of a
// source are built per this many rows), 0 if none is compiled for (k, e)
int rs_bitsliced_rows_per_wave(int k, int e);
hipError_t launch_rs_bitsliced(int k, int e, const uint8_t* src, uint8_t* out, long long pitch,
                               long long len, long long blocks, hipStream_t st, int prio = 0);
// Small batches of the single-chunk codes (16,4) (16,8) (5,4) (20,7): four
// waves per tile split the sources (k_rs_bs_split), same bytes.
bool rs_bitsliced_split_available(int k, int e);
// small-batch decode of those codes in one launch: syndromes through the
// compiled programs, the e x e solve with runtime coefficients
struct SynArgs {
    const uint8_t* src;  // [B][k] rows (erased ones never read)
    const uint8_t* par;  // [B][e] rows
    uint8_t* out;        // [B][e] rows, ascending erased order
    const uint8_t* err;  // [B][e] erased originals, strictly ascending
    int* status;         // [B]
    long long pitch, len;
};
hipError_t launch_rs_syn_split(int k, int e, const SynArgs& a, long long blocks, hipStream_t st);
hipError_t launch_rs_bitsliced_split(int k, int e, const uint8_t* src, uint8_t* out, long long pitch,
                                     long long len, long long blocks, hipStream_t st);

// Closed-form decode prepare for the gf_gen_rs_matrix code with e erased
// originals and all e parity rows surviving, per block: erasure list
// validation (strictly ascending, < k; else status -2), srcs [B][k] =
// surviving originals (ascending) then the e parity rows, dsts [B][e] = out
// rows, and the e x k decode rows V_E^-1 [V_kept | I] (no elimination) as
//   dir_addr != nullptr  k_rs_tc handler addresses [B][k][tc_rows_per_pass(e)]
//                        (e <= 32; tc_table = the context's handler table)
//   jit_coef != nullptr  the rows themselves, [B][e][k] bytes, which the
//                        emitters turn into k_rs_jit / k_rs_jitw code (e <= 63)
hipError_t launch_decode_prepare_syn(int k, int e, long long blocks, const uint8_t* err,
                                     uint8_t* out, long long out_pitch, const uint8_t** srcs,
                                     uint8_t** dsts, const unsigned long long* tc_table, int* status,
                                     const uint8_t* src, const uint8_t* par,
                                     unsigned long long* dir_addr, uint8_t* jit_coef, hipStream_t st);

// The one-matrix decode through generated code (rs_jit.hip).
struct JitArgs {
    const uint8_t* const* srcs;      // [B][k]
    uint8_t* const* dsts;            // [B][dst_stride], this launch's rows first
    const uint8_t* code;             // executable: block b, wave w, chunk ch at
                                     // code + b block_stride + (w nch + ch) chunk_stride
    long long chunk_stride;          // jit::chunk_stride(8), or jit::host_chunk_stride()
    long long block_stride;          // bytes; 0 = one program shared by every block
    int k, rows;                     // rows <= 32
    int dst_stride;                  // output pointers per block (>= rows)
    long long len;                   // % 32 == 0
    const int* status;               // [B] or nullptr (every block runs)
    int xcd_order;                   // non-zero: XCD-contiguous (block, tile) order
    int tiles_per_wg = 1;            // k_rs_jitw: column tiles per workgroup (1, 2 or 3)
    int code_prefetch = 0;           // k_rs_jitw: workgroups pull their block's code into L2 first
    int chunk_rot_ticks = 0;         // k_rs_jitw: > 0 rotates the chunk order by the start time
                                     // (s_memrealtime / chunk_rot_ticks), 0 = chunks in order
    int prio = 0;                    // k_rs_jitw / k_rs_jit: wave priority from transposes to barrier
};
// k_rs_jitw's chunk rotation period for `rows` rows at k sources: about one
// chunk's duration in 100 MHz ticks (measured best at 600 for C3's 16 rows)
int jitw_rot_ticks(int rows);
size_t jit_code_bytes(int k, int e, long long blocks);
// k_rs_jit's straight-line code (rs_jit.h) for every (block, wave, chunk) at
// code + ((b NW + w) nch + ch) jit::chunk_stride(8), from the decode rows
// coef [B][e][k] (k_decode_prepare_syn); blocks with status != 0 skipped.
hipError_t launch_jit_emit(int k, int e, long long blocks, const uint8_t* coef, const int* status,
                           uint8_t* code, hipStream_t st);
hipError_t launch_jit_fill(void* code, size_t bytes, hipStream_t st);
hipError_t launch_rs_jit(const JitArgs& a, long long blocks, hipStream_t st);
// Two waves of R rows per tile (rs_jit.h Wide): R = jitw_rows(e) (16 for
// 24 < e <= 32, 12 for 20 < e <= 24, 10 for 16 < e <= 20, else 0 = not this
// layout); code of
// block b, wave w, chunk ch at code + ((b 2 + w) nch + ch) jitw_chunk_stride(e)
int jitw_rows(int e);
// sources per chunk of that layout (rs_jit.h Wide<R, CS>)
int jitw_cs(int e);
size_t jitw_chunk_stride(int e);
size_t jitw_code_bytes(int k, int e, long long blocks);
// the wide layout covers e (16 < e <= 64 one launch; 64 < e <= 125 in passes
// of <= 64 rows, rs_jit.h wide_passes), and a pass's place in a block's code
bool jitw_layout(int e);
size_t jitw_pass_bytes(int k, int rows);
size_t jitw_pass_offset(int k, int e, int p);
hipError_t launch_jitw_emit(int k, int e, long long blocks, const uint8_t* coef, const int* status,
                            uint8_t* code, hipStream_t st);
hipError_t launch_rs_jitw(const JitArgs& a, long long blocks, hipStream_t st);
// small uploads through the kernel arguments (k_put_words): bytes % 8 == 0,
// at most sizeof(PutArgs::w)
struct PutArgs {
    static constexpr int kWords = 128;
    uint64_t w[kWords];
    uint64_t* dst;
    int n;
};
hipError_t launch_put_words(void* dst, const void* src, size_t bytes, hipStream_t st);
// device-to-device copy into executable memory (host-built code staged in
// ordinary device memory first), bytes % 8 == 0
hipError_t launch_jit_copy(void* dst, const void* src, size_t bytes, hipStream_t st);

// Threaded-code bit-sliced dot product with runtime coefficients (rs_tc.hip):
// dsts[b][i] = sum_p c_b[i][p] * srcs[b][p] for rows <= 32 per launch, where
// the coefficients arrive as handler addresses addr[b][p][slot] (slot <
// tc_rows_per_pass(rows), padding slots point at handler 0).  len % 32 == 0,
// 16-byte aligned rows; blocks with status != 0 are skipped.  More than 32
// rows run as passes of 32 (the address tables in the pass layout below).
struct TcArgs {
    const uint8_t* const* srcs;      // [B][k]
    uint8_t* const* dsts;            // [B][dst_stride], this launch's rows first
    int dst_stride;                  // row pointers per block in dsts
    const unsigned long long* addr;  // [B][k][tc_rows_per_pass(rows)]
    long long addr_stride;           // elements between blocks' tables (0: shared)
    int k, rows;
    long long len;
    const int* status;               // [B] or nullptr
};
// slots of a pass of rows <= 32: rows rounded up to 8
__host__ __device__ inline int tc_rows_per_pass(int rows) { return rows <= 0 ? 8 : (rows + 7) / 8 * 8; }
// Pass layout of a handler-address table for `rows` output rows over k
// sources: pass p (rows 32p .. 32p+31) at element offset tc_pass_offset,
// [k][tc_rows_per_pass(pass rows)] each; tc_table_elems in total.
__host__ __device__ inline int tc_passes(int rows) { return rows <= 0 ? 1 : (rows + 31) / 32; }
__host__ __device__ inline int tc_pass_rows(int rows, int p) { return rows - 32 * p < 32 ? rows - 32 * p : 32; }
__host__ __device__ inline long long tc_pass_offset(int k, int p) { return (long long)k * 32 * p; }
__host__ __device__ inline long long tc_table_elems(int k, int rows)
{
    const int np = tc_passes(rows);
    return tc_pass_offset(k, np - 1) + (long long)k * tc_rows_per_pass(tc_pass_rows(rows, np - 1));
}
// element of (output row r, source j) in a pass-layout table
__host__ __device__ inline long long tc_elem(int k, int rows, int r, int j)
{
    const int p = r / 32;
    return tc_pass_offset(k, p) + (long long)j * tc_rows_per_pass(tc_pass_rows(rows, p)) + (r & 31);
}

int tc_handler_stride();
// handlers in the table (256 per handler copy of the chained dispatch) and
// the copy serving slot s (0..7).  Consumers index the context's 2048-entry
// address table as tc_table[(slot & 7) * 256 + c]: the address of handler
// (tc_slot_copy(slot), c).
int tc_handler_count();
int tc_slot_copy(int slot);
hipError_t tc_query_handlers(unsigned long long* d_out, hipStream_t st);
hipError_t launch_rs_tc(const TcArgs& a, long long blocks, hipStream_t st);
// The same for small batches with rows <= 8 (k >= 4): four waves per tile
// split the sources, partial accumulators reduced in LDS (rs_tc.hip
// k_rs_tc_split); addr [B][k][8] as above.
hipError_t launch_rs_tc_split(const TcArgs& a, long long blocks, hipStream_t st);
// The whole one-matrix decode of a small batch in one launch (rs_tc.hip
// k_rs_tc_fused): e <= 8, 1 <= k <= 64, len % 32 == 0, 16-byte aligned rows;
// the closed-form decode rows of every block built in the kernel, status
// written per block (0, or -2 for a malformed erasure list).
struct TcFusedArgs {
    int k, e;
    long long len, pitch, blocks;
    const uint8_t* err;      // [B][e] erased originals, strictly ascending
    const uint8_t* src;      // [B][k] rows (erased ones never read)
    const uint8_t* par;      // [B][e] rows
    uint8_t* out;            // [B][e] rows
    int* status;             // [B]
    // handler of (slot s, coefficient c): map_base + (map_copy[s] 256 + c) map_stride
    unsigned long long map_base;
    int map_stride;
    int map_copy[8];
};
hipError_t launch_rs_tc_fused(const TcFusedArgs& a, hipStream_t st);

hipError_t launch_row_ptrs(const uint8_t* base, long long pitch, int rows_per_block,
                           long long blocks, const uint8_t** out, hipStream_t st);
hipError_t launch_update(const uint8_t* data, uint8_t* const* coding, const uint4* tabs4,
                         const uint32_t* ctab, int rows, long long len, hipStream_t st);

}  // namespace rsgpu
