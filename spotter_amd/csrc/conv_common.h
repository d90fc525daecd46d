// Shared pieces of the implicit-GEMM conv kernels (conv_gemm.hip: fp32 MFMA;
// conv_mfma16.hip: bf16 / 3-way-split MFMA): launch arguments and the fused epilogue.
#pragma once

#include "common.h"

namespace sp {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float act_apply(float v, int act) {
  if (act == SP_ACT_RELU) return fmaxf(v, 0.0f);
  if (act == SP_ACT_SILU) return v / (1.0f + expf(-v));
  if (act == SP_ACT_GELU) return 0.5f * v * (1.0f + erff(v * 0.70710678118654752440f));
  return v;
}

struct ConvArgs {
  sp_conv_desc d;
  int64_t M;
  int32_t K;
  int32_t HoWo;
  int32_t fast;     // Cin % 32 == 0 and 16-byte aligned operands
  int32_t vec_epi;  // 16-byte aligned C/res/scale/shift rows → float4 epilogue
  int32_t splits;   // split-K factor (>1: raw partial sums to `partial`, epilogue in splitk_reduce)
  int32_t ldp;      // row stride of a partial slab (Cout rounded up to 4)
  float* partial;   // [splits][M][ldp]
  // Batched GEMMs (the Winograd component products, winograd.hip): `batch` independent GEMMs of
  // the same shape whose A / weight planes / C start bs_a / bs_w / bs_c elements apart. Only the
  // LDS-DMA kernels (conv_glds.hip) take batch > 1; their grid is batch × tiles_per_batch.
  int32_t batch = 1;
  int32_t tiles_per_batch = 0;
  int64_t bs_a = 0, bs_w = 0, bs_c = 0;
  // A as bf16 rows (LDS-DMA kernels, bf16 operand mode only): A16 != null replaces d.A, written by the
  // producer instead of rounded per fragment in the GEMM (lda and bs_a count bf16 elements then).
  const uint16_t* A16 = nullptr;
  int64_t a_plane_stride = 0;
  // split-K with the in-launch combine (splitk_combine): one arrival counter per output tile (set by the
  // launchers whose kernels call splitk_combine, from sp_conv_desc.splitk_counters); null: the reduce launch
  int32_t* counters = nullptr;
};

// Output row offset (elements): plain row-major (out_rows_per_group == 0) or grouped rows.
__device__ __forceinline__ int64_t out_off(const sp_conv_desc& d, int64_t m) {
  if (d.out_rows_per_group <= 0) return m * d.ldc;
  const int64_t g = m / d.out_rows_per_group;
  return g * d.out_group_stride + (m - g * d.out_rows_per_group) * d.ldc;
}
__device__ __forceinline__ float* out_row(const sp_conv_desc& d, int64_t m) { return d.C + out_off(d, m); }

// bf16 activations in HBM (ABI v10: sp_conv_desc.C_bf16 / res1_bf16). bf16 → fp32 is exact; fp32 → bf16
// rounds to nearest even (v_cvt_pk_bf16_f32).
__device__ __forceinline__ float bf16_lo(uint32_t u) { return __builtin_bit_cast(float, u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __builtin_bit_cast(float, u & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b2));
}

// BF (template flag of the epilogue helpers below): the kernel may see bf16 rows (the bf16 operand mode's
// kernels); the fp32-only kernels instantiate BF = false and carry no bf16 branches (sp_conv2d refuses bf16
// rows outside the bf16 operand mode).
// The res1 row segment n..n+3 of row m (fp32 or bf16 residual rows), zero without a residual.
template <bool BF = false>
__device__ __forceinline__ float4 load_res1(const sp_conv_desc& d, int64_t m, int n) {
  if (BF && d.res1_bf16) {
    const uint2 u = *reinterpret_cast<const uint2*>(d.res1_bf16 + m * d.ldr1 + n);
    return make_float4(bf16_lo(u.x), bf16_hi(u.x), bf16_lo(u.y), bf16_hi(u.y));
  }
  if (d.res1) return *reinterpret_cast<const float4*>(d.res1 + m * d.ldr1 + n);
  return make_float4(0.f, 0.f, 0.f, 0.f);
}
template <bool BF = false>
__device__ __forceinline__ bool has_res1(const sp_conv_desc& d) { return d.res1 || (BF && d.res1_bf16); }

// Store the finished float4 of row m, channels n..n+3 (fp32 rows or bf16 rows).
template <bool BF = false>
__device__ __forceinline__ void store_out4(const sp_conv_desc& d, int64_t m, int n, float4 v) {
  if (BF && d.C_bf16) {
    *reinterpret_cast<uint2*>(d.C_bf16 + out_off(d, m) + n) = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
  } else {
    *reinterpret_cast<float4*>(out_row(d, m) + n) = v;
  }
}

// The fused epilogue on four consecutive output channels n..n+3 of row m (p.vec_epi, n+3 < Cout),
// with the res1 row segment already loaded (r1; ignored when d.res1 is null).
template <bool BF = false>
__device__ __forceinline__ void epilogue_vec(const ConvArgs& p, int64_t m, int n, float4 v, float4 r1) {
  const sp_conv_desc& d = p.d;
  if (d.row_scale) {
    const float rs = d.row_scale[m % d.row_period];
    v.x *= rs; v.y *= rs; v.z *= rs; v.w *= rs;
  }
  const float4 sc = d.scale ? *reinterpret_cast<const float4*>(d.scale + n) : make_float4(1.f, 1.f, 1.f, 1.f);
  const float4 sh = d.shift ? *reinterpret_cast<const float4*>(d.shift + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  v.x = fmaf(v.x, sc.x, sh.x); v.y = fmaf(v.y, sc.y, sh.y);
  v.z = fmaf(v.z, sc.z, sh.z); v.w = fmaf(v.w, sc.w, sh.w);
  if (has_res1<BF>(d)) {
    v.x += r1.x; v.y += r1.y; v.z += r1.z; v.w += r1.w;
  }
  v.x = act_apply(v.x, d.act); v.y = act_apply(v.y, d.act);
  v.z = act_apply(v.z, d.act); v.w = act_apply(v.w, d.act);
  if (d.res2) {
    const float4 a = *reinterpret_cast<const float4*>(d.res2 + m * d.ldr2 + n);
    v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
  } else if (BF && d.res2_bf16) {
    const uint2 u = *reinterpret_cast<const uint2*>(d.res2_bf16 + m * d.ldr2 + n);
    v.x += bf16_lo(u.x); v.y += bf16_hi(u.x); v.z += bf16_lo(u.y); v.w += bf16_hi(u.y);
  }
  store_out4<BF>(d, m, n, v);
}

// The fused epilogue on four consecutive output channels n..n+3 of row m.
template <bool BF = false>
__device__ __forceinline__ void epilogue_store(const ConvArgs& p, int64_t m, int n, float4 v) {
  const sp_conv_desc& d = p.d;
  SP_BCHECK(m, p.M);
  SP_BCHECK(n, d.Cout);
  if (p.vec_epi && n + 3 < d.Cout) {
    epilogue_vec<BF>(p, m, n, v, load_res1<BF>(d, m, n));
  } else {
    const int64_t ro = out_off(d, m);
    float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int nn = n + u;
      if (nn >= d.Cout) break;
      float x = e[u];
      if (d.row_scale) x *= d.row_scale[m % d.row_period];
      x = fmaf(x, d.scale ? d.scale[nn] : 1.0f, d.shift ? d.shift[nn] : 0.0f);
      if (d.res1) x += d.res1[m * d.ldr1 + nn];
      if (BF && d.res1_bf16) x += bf16_lo(d.res1_bf16[m * d.ldr1 + nn]);
      x = act_apply(x, d.act);
      if (d.res2) x += d.res2[m * d.ldr2 + nn];
      if (BF && d.res2_bf16) x += bf16_lo(d.res2_bf16[m * d.ldr2 + nn]);
      if (BF && d.C_bf16) d.C_bf16[ro + nn] = (uint16_t)(pack_bf16x2(x, 0.f) & 0xffffu);
      else d.C[ro + nn] = x;
    }
  }
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// A buffer descriptor over the split-K partial slabs (offsets below 2^31 bytes: splitk_counters_for).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t partial_rsrc(const ConvArgs& p) {
  return __builtin_amdgcn_make_buffer_rsrc(p.partial, 0, 0x7fffffff, 0x00020000);
}

// One float4 of this workgroup's split-K partial slab (z = blockIdx.z). With the in-launch combine
// (p.counters) the store is write-through (sc1), so the tile's last workgroup, on any CU or XCD, reads it with
// sc1 loads and no agent release / acquire fence is needed (cdna_hip_programming.md §6 Guideline 16 R1).
// CNT: compiled only into the kernels that take counters (conv_mfma16_kernel, conv_gemm_kernel); every other
// kernel keeps the plain store and never reads p.counters (no extra SGPRs in their epilogues).
template <bool CNT = false>
__device__ __forceinline__ void store_partial(const ConvArgs& p, int64_t m, int n, float4 v) {
  const int64_t e = ((int64_t)blockIdx.z * p.M + m) * p.ldp + n;
  SP_BCHECK(e + 3, p.d.workspace_elems);  // the split-K slabs [splits][M][ldp] fit the caller's workspace
  SP_BCHECK(m, p.M);
  if (CNT && p.counters)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), partial_rsrc(p), (int)(e * 4), 0, 16);
  else
    *reinterpret_cast<float4*>(p.partial + e) = v;
}

// Accumulator band i of a wave (TN 32x32 MFMA tiles, v_mfma_f32_32x32x*: lane (r, h) holds
// rows (q&3) + 8(q>>2) + 4h, column r) → the wave's private LDS slab → fused epilogue on
// float4s of one output row (or raw partial sums for split-K).
template <int TN, bool BF = false, bool CNT = false>
__device__ __forceinline__ void epilogue_band(const ConvArgs& p, float* slab, const f32x16* accrow,
                                              int64_t mb, int nb, int lane) {
  constexpr int WN = TN * 32;
  const int r = lane & 31;
  const int h = lane >> 5;
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) slab[((q & 3) + 8 * (q >> 2) + 4 * h) * WN + j * 32 + r] = accrow[j][q];
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes done
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int t = 0; t < (32 * WN / 4) / 64; ++t) {
    const int c = lane + 64 * t;
    const int row = c / (WN / 4);
    const int col = (c - row * (WN / 4)) * 4;
    const int64_t m = mb + row;
    const int n = nb + col;
    if (m >= p.M || n >= p.d.Cout) continue;
    float4 v = *reinterpret_cast<const float4*>(slab + row * WN + col);
    if (p.splits > 1) {
      store_partial<CNT>(p, m, n, v);
    } else {
      epilogue_store<BF>(p, m, n, v);
    }
  }
  __builtin_amdgcn_wave_barrier();
}

// The TM accumulator bands of a wave → its LDS region (NB bands of 32 × 32TN floats at a time),
// then the fused epilogue on float4s of one output row, with the res1 loads of G consecutive
// tasks issued before their stores so the residual fetch latency overlaps. NB = TM when the
// region fits in the operand stages' LDS, else 1 (band by band).
// L16: the f32x16 of each 32×32 block holds 2×2 blocks of v_mfma_f32_16x16x32 results (element
// q = 8·bi + 4·bj + reg; lane l holds rows 16bi + 4(l >> 4) + reg, column 16bj + (l & 15)).
template <int TM, int TN, int NB, bool L16 = false, bool BF = false, bool CNT = false>
__device__ __forceinline__ void epilogue_tile(const ConvArgs& p, float* region, f32x16 (*acc)[TN],
                                              int64_t mb, int nb, int lane) {
  static_assert(TM % NB == 0, "bands per round must divide TM");
  constexpr int WN = TN * 32;
  constexpr int PER = NB * (32 * WN / 4) / 64;  // float4 tasks per lane per round
  constexpr int G = PER < 4 ? PER : 4;
  static_assert(PER % G == 0, "task groups");
  const int r = lane & 31;
  const int h = lane >> 5;
  const sp_conv_desc& d = p.d;
  const bool fastv = p.vec_epi && p.splits == 1;
#pragma unroll
  for (int i0 = 0; i0 < TM; i0 += NB) {
    if (i0) __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int rr = L16 ? 16 * (q >> 3) + 4 * (lane >> 4) + (q & 3) : (q & 3) + 8 * (q >> 2) + 4 * h;
          const int cc = L16 ? 16 * ((q >> 2) & 1) + (lane & 15) : r;
          region[(i * 32 + rr) * WN + j * 32 + cc] = acc[i0 + i][j][q];
        }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    const int64_t mr = mb + i0 * 32;
    for (int t0 = 0; t0 < PER; t0 += G) {
      float4 r1[G];
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int cidx = lane + 64 * (t0 + u);
        const int row = cidx / (WN / 4);
        const int col = (cidx - row * (WN / 4)) * 4;
        const int64_t m = mr + row;
        const int n = nb + col;
        r1[u] = (fastv && has_res1<BF>(d) && m < p.M && n < d.Cout) ? load_res1<BF>(d, m, n) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int cidx = lane + 64 * (t0 + u);
        const int row = cidx / (WN / 4);
        const int col = (cidx - row * (WN / 4)) * 4;
        const int64_t m = mr + row;
        const int n = nb + col;
        if (m >= p.M || n >= d.Cout) continue;
        const float4 v = *reinterpret_cast<const float4*>(region + row * WN + col);
        if (p.splits > 1) {
          store_partial<CNT>(p, m, n, v);
        } else if (fastv) {
          epilogue_vec<BF>(p, m, n, v, r1[u]);
        } else {
          epilogue_store<BF>(p, m, n, v);
        }
      }
    }
  }
}

// The counters a split-K launch of `tiles` output tiles may use: the descriptor's array when it has one
// entry per tile (and the partial slabs are addressable by 32-bit buffer offsets, at most 16 splits), else
// null (the separate reduce launch).
inline int32_t* splitk_counters_for(const ConvArgs& a, int64_t tiles) {
  return (a.splits > 1 && a.splits <= 16 && a.d.splitk_counters && tiles <= a.d.splitk_counters_len &&
          (int64_t)a.splits * a.M * a.ldp * 4 < (int64_t(1) << 31))
             ? a.d.splitk_counters
             : nullptr;
}

// In-launch split-K combine (ABI v13), called by every workgroup of a split-K launch with counters after its
// partial tile went out (store_partial: write-through sc1 stores). The hand-off follows the MI355X guide
// (cdna_hip_programming.md §5 "In-launch split-K reduction", its sc1 form; §6 Guideline 16 R1): every wave
// drains its stores, the workgroup meets at a barrier, one lane draws a ticket (relaxed agent-scope add);
// the workgroup that draws splits − 1 resets the counter for the next launch and combines the tile with sc1
// loads (no acquire fence): Σ_z partial[z] in z order, then the epilogue — splitk_reduce_kernel's arithmetic,
// so the output is bit-identical to the two-launch form. Each thread keeps 16 partial loads in flight (its
// TPT float4 tasks × 16 / TPT splits per round) beside its residual loads. `flag` is a word of the kernel's one LDS array (no second __shared__ object), free
// once the epilogue is done.
template <int NT, int BM, int BN>
__device__ __forceinline__ void splitk_combine(const ConvArgs& p, int* flag, int tile, int64_t m0, int n0) {
  constexpr int TPT = BM * BN / 4 / NT;  // float4 tasks per thread
  static_assert(TPT * NT * 4 == BM * BN && TPT <= 16, "combine tasks");
  constexpr int ZB = 16 / TPT;           // splits loaded per round: TPT · ZB = 16 loads in flight
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its write-through partial stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(p.counters + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == p.splits - 1;
    if (last) __hip_atomic_store(p.counters + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  const __amdgpu_buffer_rsrc_t rs = partial_rsrc(p);
  const int zs = (int)(p.M * p.ldp * 4);  // bytes between split slabs
  const sp_conv_desc& d = p.d;
  int64_t mm[TPT];
  int nn[TPT], off[TPT];
  bool ok[TPT];
  float4 v[TPT], r1[TPT];
#pragma unroll
  for (int t = 0; t < TPT; ++t) {
    const int i = threadIdx.x + NT * t;
    const int row = i / (BN / 4);
    mm[t] = m0 + row;
    nn[t] = n0 + (i - row * (BN / 4)) * 4;
    ok[t] = mm[t] < p.M && nn[t] < d.Cout;
    off[t] = ok[t] ? (int)((mm[t] * p.ldp + nn[t]) * 4) : 0;
    // the residual segment in flight with the partials (epilogue_vec's operand)
    r1[t] = (ok[t] && p.vec_epi && nn[t] + 3 < d.Cout) ? load_res1(d, mm[t], nn[t]) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  for (int z0 = 0; z0 < p.splits; z0 += ZB) {
    u32x4 u[TPT][ZB];
#pragma unroll
    for (int j = 0; j < ZB; ++j)
      if (z0 + j < p.splits)
#pragma unroll
        for (int t = 0; t < TPT; ++t) u[t][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, off[t] + (z0 + j) * zs, 0, 16);
#pragma unroll
    for (int j = 0; j < ZB; ++j)
      if (z0 + j < p.splits)
#pragma unroll
        for (int t = 0; t < TPT; ++t) {
          const float4 w = __builtin_bit_cast(float4, u[t][j]);
          if (z0 + j == 0) {
            v[t] = w;
          } else {
            v[t].x += w.x; v[t].y += w.y; v[t].z += w.z; v[t].w += w.w;
          }
        }
  }
#pragma unroll
  for (int t = 0; t < TPT; ++t) {
    if (!ok[t]) continue;
    if (p.vec_epi && nn[t] + 3 < d.Cout) epilogue_vec(p, mm[t], nn[t], v[t], r1[t]);
    else epilogue_store(p, mm[t], nn[t], v[t]);
  }
}

// Row-LayerNorm epilogue (sp_conv_desc.ln_gamma): the workgroup holds whole output rows — BM = 32 rows
// × BN = Cout columns, 4 waves side by side along N, each wave's 32 × 32·TN accumulators (v_mfma_f32_32x32x*
// layout) — staged in LDS, then one wave per row: bias / BN affine, residual, two-pass mean and variance
// over the row (the sp_layernorm arithmetic), gamma / beta, 4-byte-per-lane coalesced stores.
template <int TN>
__device__ __forceinline__ void epilogue_rowln(const ConvArgs& p, float* tile, const f32x16* acc, int64_t m0,
                                               int wave, int lane) {
  constexpr int BN = 128 * TN;
  constexpr int LDT = BN + 4;
  constexpr int PER = BN / 64;
  const int r = lane & 31;
  const int h = lane >> 5;
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) tile[((q & 3) + 8 * (q >> 2) + 4 * h) * LDT + wave * 32 * TN + j * 32 + r] = acc[j][q];
  __syncthreads();
  const sp_conv_desc& d = p.d;
  const int N = d.Cout;
  for (int rr = wave; rr < 32; rr += 4) {
    const int64_t m = m0 + rr;
    if (m >= p.M) break;
    const float rs = d.row_scale ? d.row_scale[m % d.row_period] : 1.0f;
    float v[PER];
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = lane + 64 * u;
      float x = 0.f;
      if (c < N) {
        x = fmaf(tile[rr * LDT + c] * rs, d.scale ? d.scale[c] : 1.0f, d.shift ? d.shift[c] : 0.0f);
        if (d.res1) x += d.res1[m * d.ldr1 + c];
      }
      v[u] = x;
      s += x;
    }
    const float mean = wave_sum(s) / (float)N;
    float q = 0.f;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = lane + 64 * u;
      const float t = c < N ? v[u] - mean : 0.f;
      q += t * t;
    }
    const float var = wave_sum(q) / (float)N;
    const float rstd = 1.0f / sqrtf(var + d.ln_eps);
    float* orow = out_row(d, m);
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = lane + 64 * u;
      if (c < N) orow[c] = (v[u] - mean) * rstd * d.ln_gamma[c] + d.ln_beta[c];
    }
  }
}

// conv_mfma16.hip: bf16-operand MFMA GEMM (planes = 1: bf16; planes = 3: fp32 via a 3-way bf16
// split). cfg < 0 picks the tile by shape. Returns 0 or the launch error.
int launch_mfma16(const ConvArgs& a, int planes, int cfg, hipStream_t s);
// The LDS-DMA tile configurations of launch_mfma16 (conv_glds.hip); -2 when cfg is not one of them.
int launch_glds_cfg(const ConvArgs& a, int planes, int cfg, hipStream_t s);
// Tuning: the split mode's slab-epilogue form for the calling thread (4 = direct stores, else the slab
// store pass; sp_set_tuning SP_TUNE_GLDS_EPILOGUE).
void set_glds_epilogue(int v);
// The tile configuration sp_set_conv_config forced for the calling thread (-1: none).
int forced_cfg();
// Split-K combine kernel launch (conv_gemm.hip).
int launch_splitk_reduce(const ConvArgs& a, hipStream_t s);

}  // namespace sp
