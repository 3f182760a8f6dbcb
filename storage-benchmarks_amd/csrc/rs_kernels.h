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

struct PrepArgs {
    int k, e, rows_pad;
    long long blocks;
    const uint8_t* err;           // device [blocks][e]
    const uint8_t* src; long long src_pitch;
    const uint8_t* par; long long par_pitch;
    uint8_t* out; long long out_pitch;
    const uint8_t** surv_ptrs;    // device [blocks][k]
    uint8_t** out_ptrs;           // device [blocks][e]
    uint4* tabs4; uint32_t* ctab; long long tab_block_stride;  // v_perm tables, or nullptr
    int* status;                  // device [blocks]
    // k_rs_tc instead of k_dot_generic (when non-null): the context's
    // 512-entry handler table and the [blocks][k][tc_rows] address output
    const unsigned long long* tc_table = nullptr;
    unsigned long long* tc_addr = nullptr;
    int tc_rows = 0;
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
// Bit-sliced RS(k, e) with compile-time coefficients (rs_bitsliced.hip).
// emask == nullptr: parity of the gf_gen_rs_matrix code into `out`.
// emask != nullptr ([blocks][2] bitmask of erased originals): syndromes
//   out[p] = par[p] ^ sum_{j not erased} 2^(p j) src[j].
// Requires len % 32 == 0, 16-byte aligned rows.
bool rs_bitsliced_available(int k, int e);
hipError_t launch_rs_bitsliced(int k, int e, const uint8_t* src, const uint8_t* par, uint8_t* out,
                               long long pitch, long long len, long long blocks,
                               const uint64_t* emask, hipStream_t st);

// Syndrome-decode prepare: per block, emask, V_E^-1 and its consumers' tables:
// k_dot_generic tables (tabs4/ctab, when non-null) and/or k_rs_tc handler
// addresses (tc_addr [B][e][tc_rows], when non-null; tc_table = the 256
// handler addresses).  syn_addr (non-null with tc_table): [B][k-e][tc_rows]
// handler addresses of the syndrome rows 2^(r j) per surviving original j
// (ascending), for the fused decode's threaded-code syndrome phase.
// dir_addr (non-null with tc_table): the one-matrix decode through k_rs_tc --
// srcs [B][k] = surviving originals (ascending) then the e parity rows (from
// src / par), dsts [B][e] = out rows, dir_addr [B][k][tc_rows] = handler
// addresses of the e x k decode rows V_E^-1 [V_kept | I].
hipError_t launch_decode_prepare_syn(int k, int e, int rows_pad, long long blocks,
                                     const uint8_t* err, uint8_t* out, long long out_pitch,
                                     const uint8_t** srcs, uint8_t** dsts, uint4* tabs4,
                                     uint32_t* ctab, long long tab_block_stride,
                                     const unsigned long long* tc_table,
                                     unsigned long long* tc_addr, int tc_rows,
                                     unsigned long long* emask, int* status,
                                     unsigned long long* syn_addr, const uint8_t* src,
                                     const uint8_t* par, unsigned long long* dir_addr,
                                     hipStream_t st);

// Threaded-code bit-sliced dot product with runtime coefficients (rs_tc.hip):
// dsts[b][i] = sum_p c_b[i][p] * srcs[b][p] for rows <= 32, where the
// coefficients arrive as handler addresses addr[b][p][slot] (slot < tc_rows,
// padding slots point at handler 0).  len % 32 == 0, 16-byte aligned rows;
// blocks with status != 0 are skipped.
struct TcArgs {
    const uint8_t* const* srcs;      // [B][k]
    uint8_t* const* dsts;            // [B][rows]
    const unsigned long long* addr;  // [B][k][tc_rows_per_pass(rows)]
    long long addr_stride;           // elements between blocks' tables (0: shared)
    int k, rows;
    long long len;
    const int* status;               // [B] or nullptr
};
int tc_rows_per_pass(int rows);

// One-pass syndrome decode (rs_decode_fused.hip) for the instantiated
// gf_gen_rs_matrix codes: out[b] = data rows listed by the prepare kernel's
// emask, from src (surviving data) and par; addr = k_rs_tc handler addresses
// of V_E^-1 ([B][e][tc_rows_per_pass(e)]); blocks with status != 0 skipped.
bool rs_decode_fused_available(int k, int e);
hipError_t launch_rs_decode_fused(int k, int e, const uint8_t* src, const uint8_t* par,
                                  uint8_t* out, long long pitch, long long len, long long blocks,
                                  const uint64_t* emask, const unsigned long long* addr,
                                  const unsigned long long* syn_addr, const int* status,
                                  hipStream_t st);
int tc_handler_stride();
// handlers in the table (256 per handler copy of the chained dispatch) and
// the copy serving slot s (0..7).  Consumers index the context's 2048-entry
// address table as tc_table[(slot & 7) * 256 + c]: the address of handler
// (tc_slot_copy(slot), c).
int tc_handler_count();
int tc_slot_copy(int slot);
hipError_t tc_query_handlers(unsigned long long* d_out, hipStream_t st);
hipError_t launch_rs_tc(const TcArgs& a, long long blocks, hipStream_t st);

hipError_t launch_row_ptrs(const uint8_t* base, long long pitch, int rows_per_block,
                           long long blocks, const uint8_t** out, hipStream_t st);
hipError_t launch_update(const uint8_t* data, uint8_t* const* coding, const uint4* tabs4,
                         const uint32_t* ctab, int rows, long long len, hipStream_t st);

}  // namespace rsgpu
