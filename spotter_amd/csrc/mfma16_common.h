// Pieces shared by the bf16-operand MFMA GEMM kernels (conv_mfma16.hip, conv_glds.hip): the bf16 /
// 3-way split operand forms, the six-product MFMA sums and the LDS-DMA primitives.
#pragma once

#include "conv_common.h"

namespace sp {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int KT = 32;  // k per LDS stage

__device__ __forceinline__ int sw16(int row, int c) { return row * 4 + (c ^ ((row >> 2) & 3)); }

// 8 fp32 → PL bf16 planes (RNE). PL = 3: exact residual chain hi / mid / lo.
template <int PL>
__device__ __forceinline__ void split8(const float4& x0, const float4& x1, bf16x8* out) {
  const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
  bf16x8 h, m, l;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    h[j] = (__bf16)v[j];
    if constexpr (PL == 3) {
      const float r1 = v[j] - (float)h[j];
      m[j] = (__bf16)r1;
      const float r2 = r1 - (float)m[j];
      l[j] = (__bf16)r2;
    }
  }
  out[0] = h;
  if constexpr (PL == 3) {
    out[1] = m;
    out[2] = l;
  }
}

template <int PL>
__device__ __forceinline__ f32x16 mfma_planes(const bf16x8* a, const bf16x8* b, f32x16 acc) {
  if constexpr (PL == 1) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  } else {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  }
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Same six-product sum on v_mfma_f32_16x16x32_bf16 (one 16×16 block, k = 32 per instruction).
template <int PL>
__device__ __forceinline__ f32x4 mfma16x16_planes(const bf16x8* a, const bf16x8* b, f32x4 acc) {
  if constexpr (PL == 1) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
  } else {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
  }
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA pipelined variant (no A2 addend, Cin % 32 == 0): every operand byte goes global → LDS
// by global_load_lds_dwordx4 (16 B per lane, no VGPR round trip), NS stages deep, one raw
// s_barrier per k-tile and a counted vmcnt that keeps NS-2 stages in flight across it. A is staged
// as raw fp32 (the k-tile's 32 channels = 8 × 16-byte chunks per im2col row) and split into bf16
// planes by each wave at fragment-read time, so the split VALU work interleaves with the MFMAs of
// the same wave instead of sitting between the load wait and the barrier. The DMA destination is
// lane-linear (wave base + 16·lane), so the bank swizzle is applied on the SOURCE side: LDS chunk
// position q of A row r holds global chunk q ^ ((r >> 1) & 7) (conflict-free b128 fragment reads,
// the fp32 kernel's swizzle), position q of a B row holds chunk q ^ ((r >> 2) & 3) (sw16).
// Padding taps, rows past M and columns past Cout read a 128-byte zero block instead.
__device__ float4 g_zero_chunk[16];  // 256 B: the widest staged row chunk offset (fp32 A at BK = 64) stays inside

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Two fp32 → one packed bf16 pair (RNE): a single v_cvt_pk_bf16_f32.
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  const f32x2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

// split8 written pair by pair so it compiles to the minimum VALU stream per 8 elements: 12
// v_cvt_pk_bf16_f32, 8 + 8 unpacks (the low half of a pair is `u << 16`, the high half `u &
// 0xffff0000`: bf16 → fp32 is exact) and 16 v_sub_f32 — 44 instructions, against ~60 for the
// element-wise form (hipcc converts element by element, then repacks). Same RNE hi / mid / lo as split8.
// Round 5 built the residual subtractions as packed pairs (f32x2 arithmetic → v_pk_add_f32: 36 VALU per 8
// elements instead of 44, bit-identical); it measured 0.3 % slower in the C2 step (same box, alternating,
// profiles/r5/x3/ab_round5_changes.json), so the scalar form stays. -DSP_SPLIT_PK2=1: the packed form (A/B).
#ifndef SP_SPLIT_PK2
#define SP_SPLIT_PK2 0
#endif
template <int PL>
__device__ __forceinline__ void split_frag_pk(const float4& x0, const float4& x1, bf16x8* out) {
  const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
  uint32_t H[4], M[4], L[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float a = v[2 * q], b = v[2 * q + 1];
    const uint32_t h = cvt_pk_bf16(a, b);
    H[q] = h;
    if constexpr (PL == 3) {
#if SP_SPLIT_PK2
      const f32x2 ab = {a, b};
      const f32x2 hf = {__builtin_bit_cast(float, h << 16), __builtin_bit_cast(float, h & 0xffff0000u)};
      const f32x2 r = ab - hf;
      const uint32_t m = cvt_pk_bf16(r.x, r.y);
      M[q] = m;
      const f32x2 mf = {__builtin_bit_cast(float, m << 16), __builtin_bit_cast(float, m & 0xffff0000u)};
      const f32x2 r2 = r - mf;
      L[q] = cvt_pk_bf16(r2.x, r2.y);
#else
      const float ra = a - __builtin_bit_cast(float, h << 16);
      const float rb = b - __builtin_bit_cast(float, h & 0xffff0000u);
      const uint32_t m = cvt_pk_bf16(ra, rb);
      M[q] = m;
      L[q] = cvt_pk_bf16(ra - __builtin_bit_cast(float, m << 16), rb - __builtin_bit_cast(float, m & 0xffff0000u));
#endif
    }
  }
  out[0] = __builtin_bit_cast(bf16x8, make_uint4(H[0], H[1], H[2], H[3]));
  if constexpr (PL == 3) {
    out[1] = __builtin_bit_cast(bf16x8, make_uint4(M[0], M[1], M[2], M[3]));
    out[2] = __builtin_bit_cast(bf16x8, make_uint4(L[0], L[1], L[2], L[3]));
  }
}

template <int PL>
__device__ __forceinline__ void split_frag(const float4& x0, const float4& x1, bf16x8* out) {
  split_frag_pk<PL>(x0, x1, out);
}

// s_waitcnt vmcnt(n) with expcnt / lgkmcnt left open (gfx9 encoding; n < 64), fenced for the
// compiler so no LDS access moves across it.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  asm volatile("" ::: "memory");
}

// Raw s_barrier (no implied vmcnt(0), unlike __syncthreads), fenced for the compiler.
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// One global_load_lds_dwordx4: 16 bytes from each lane's gsrc to LDS byte address
// lds_base + 16·lane (lds_base wave-uniform). Issued as inline asm so hipcc does not track it:
// the builtin form makes hipcc wait vmcnt(0) before every later ds_read of the same array, which
// drains the stage pipeline; completion is counted by hand (wait_vmcnt + raw_barrier).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_base)
      : "memory");
}

// The same DMA with a wave-uniform 64-bit base in SGPRs and a 32-bit per-lane byte offset
// (global_load_lds_dwordx4 vOff, s[base]): advancing a k-step is then one scalar add on the base
// instead of a 64-bit VALU add + bounds select per piece (the 1×1 / batched-GEMM fast path).
__device__ __forceinline__ void glds16s(uint32_t voff, const void* base, uint32_t lds_base) {
  // the base IS wave-uniform, but hipcc cannot always prove it (it then hands the "s" operand a
  // VGPR pair, which the assembler rejects): pin it to SGPRs
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  const uint64_t sbase = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds_base)
      : "memory");
}

// XCD-aware bijective remap of a 1-D grid: MI355X deals consecutive workgroups round-robin over the
// 8 XCDs, so workgroup b runs on XCD b % 8; index v gives each XCD a contiguous run.
__device__ __forceinline__ int xcd_index(int b, int nwg) {
  const int xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
}

}  // namespace
}  // namespace sp
