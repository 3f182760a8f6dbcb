// jit_prog.h -- host-built generated code for a coefficient matrix shared by
// every block (the runtime-coefficient encode: caller `coef`, Cauchy,
// ec_encode_data's gftbls, codes without a compile-time kernel).
//
// The code runs in k_rs_jit (rs_jit.hip) exactly like the per-block decode
// code, with the register contract of rs_jit.h, but each (wave, source)
// preamble builds only the composites its 64 masks need: a greedy cover
// (the algorithm of gen_enc_progs.py, which serves the compile-time encode)
// picks XORs of 2 or 3 available values until every mask is the XOR of at
// most two values, so the multiply-accumulate stays one instruction per
// output plane.  13.4 composites per source for random coefficients against
// the 22 of the full four-Russians tables; when a cover would need more than
// 22, the full tables serve.  Everything here runs on the host: the matrix
// is known there, and the code is built once per matrix and cached.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <utility>
#include <vector>

namespace rsgpu {
namespace jit {

constexpr int kMaxComposites = 22;  // v32..v53
constexpr uint8_t kNone = 255;

constexpr int kMaxSlots = 16;       // rows per wave: 8 (k_rs_jit), up to 16 (k_rs_jitw)

// One (wave, source) program: value ids 0..7 are the source's planes
// (bit i of a mask = plane i), 8 + i the composite ops[i] = XOR of its 2 or 3
// operand values; accumulator plane b of slot s gets outs[8 s + b] (0, 1 or
// 2 values) XORed in.
struct SrcProg {
    int nops = 0;
    uint8_t ops[kMaxComposites][3];
    uint8_t outs[8 * kMaxSlots][2];
};

// Cover of the masks of coefficients coef[0..nslot-1] (slot s = output row
// R w + s of the wave), nslot <= kMaxSlots.
void plan_source(const uint8_t* coef, int nslot, SrcProg& p, int max_ops = kMaxComposites);

// Largest chunk (8 sources, 8 slots, kMaxComposites 3-input composites),
// rounded to 64-byte lines: the stride between chunks of host-built code.
int host_chunk_stride();

// Code of one chunk (nt <= 8 sources with programs progs[0..nt-1], nslot <=
// 8 slots) at dst; returns its size in bytes (<= host_chunk_stride()).
size_t emit_chunk(uint8_t* dst, int nt, int nslot, const SrcProg* progs);

// The whole program of an e x k matrix c (row-major) in passes of <= 32
// rows: pass p, wave w, chunk ch at ((p NW_MAX + w) nch + ch) stride, with
// NW_MAX = 4 wave slots reserved per pass.  Returns the bytes.
// max_ops < kMaxComposites caps the greedy cover (tests use it to exercise
// the full-table fallback).
std::vector<uint8_t> build_matrix_code(const uint8_t* c, int k, int e, int* chunk_stride,
                                       int max_ops = kMaxComposites);

// The same in the two-wave layout of k_rs_jitw (rs_jit.h Wide<R, CS>, the
// register contract of the decode: planes v10..v17, composites v18..v39,
// accumulators from v40, LDS address in v9) for 16 < e <= 32: wave w (rows
// R w .. R w + R - 1), chunk ch of CS sources at (w nch + ch) stride, each
// source loading its own planes, then its covered composites and one
// instruction per nonzero output mask.  *chunk_stride = the largest chunk
// rounded to 64 bytes.
std::vector<uint8_t> build_matrix_code_wide(const uint8_t* c, int k, int e, int R, int CS, int* chunk_stride,
                                            int max_ops = kMaxComposites);

// Rows of any count the wide layout takes (16 < e <= 125): passes of <= 64
// rows (rs_jit.h wide_passes), each built as above in the layout of its own
// row count (jitw_rows / jitw_cs) and appended; passes[p] = (byte offset of
// pass p, its chunk stride).  Empty when a pass fits no layout.  The
// GENERATED encode's shared programs (rsgpu_capi.cpp shared_program) are
// exactly this.
std::vector<uint8_t> build_matrix_code_wide_passes(const uint8_t* c, int k, int e,
                                                   std::vector<std::pair<size_t, int>>* passes,
                                                   int max_ops = kMaxComposites);

}  // namespace jit
}  // namespace rsgpu
