// Implicit-GEMM convolution / linear layer on fp32 MFMA (gfx950).
//
// One kernel covers every conv and nn.Linear on the RT-DETRv2 path: the
// ResNet-vd backbone (RN:38-68, RN:179-231), encoder input projections
// (M2:1350-1360), CCFM convs (M2:817-835, M2:907-952), AIFI / decoder
// projections and FFNs (M2:228-242, M2:273-336), MSDA value/offset/weight/
// output projections (M2:144-147) and the heads (M2:1376-1381, M2:1777-1787).
//
// Math: out[m, n] = epilogue(Σ_k A[m, k] · W[n, k]) with A gathered on the fly
// from NHWC activations (im2col never materialised) and W stored [Cout][K]
// (k contiguous). Tile BM×BN×32 per 256-thread workgroup (2×2 waves), each
// wave a (32·TM)×(32·TN) patch of v_mfma_f32_32x32x2f32 accumulators (exact
// fp32 fmaf chains, 64 FLOP/clk/SIMD). A and B tiles are staged through LDS as
// row-major [row][32 k] with a 16-byte-chunk XOR swizzle so the per-lane
// ds_read_b128 fragment reads are conflict-free; the k order inside an 8-deep
// slab is permuted (lane half h owns k = 8s + 4h + j) identically for A and B,
// which lets one ds_read_b128 feed four MFMAs. Global loads for tile t+1 are
// issued before the MFMAs of tile t (register staging).
//
// Epilogue (fused): row mask (query-selection valid_mask, M2:1592), per-channel
// BatchNorm scale/shift (FrozenBN M2:748-758 / eval BN), residual, activation,
// post-activation residual, and a grouped output row map so projections write
// straight into concatenated / flattened buffers (M2:1553-1555).
#include <cstdlib>

#include "common.h"

namespace sp {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;

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
};

// The fused epilogue on four consecutive output channels n..n+3 of row m.
__device__ __forceinline__ void epilogue_store(const ConvArgs& p, int64_t m, int n, float4 v) {
  const sp_conv_desc& d = p.d;
  const int rpg = d.out_rows_per_group > 0 ? d.out_rows_per_group : 0x7fffffff;
  const int64_t g = m / rpg;
  const int64_t rr = m - g * rpg;
  float* crow = d.C + g * d.out_group_stride + rr * d.ldc;
  if (p.vec_epi && n + 3 < d.Cout) {
    if (d.row_scale) {
      const float rs = d.row_scale[m % d.row_period];
      v.x *= rs; v.y *= rs; v.z *= rs; v.w *= rs;
    }
    float4 sc = d.scale ? *reinterpret_cast<const float4*>(d.scale + n) : make_float4(1.f, 1.f, 1.f, 1.f);
    float4 sh = d.shift ? *reinterpret_cast<const float4*>(d.shift + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    v.x = fmaf(v.x, sc.x, sh.x); v.y = fmaf(v.y, sc.y, sh.y);
    v.z = fmaf(v.z, sc.z, sh.z); v.w = fmaf(v.w, sc.w, sh.w);
    if (d.res1) {
      float4 a = *reinterpret_cast<const float4*>(d.res1 + m * d.ldr1 + n);
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    v.x = act_apply(v.x, d.act); v.y = act_apply(v.y, d.act);
    v.z = act_apply(v.z, d.act); v.w = act_apply(v.w, d.act);
    if (d.res2) {
      float4 a = *reinterpret_cast<const float4*>(d.res2 + m * d.ldr2 + n);
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    *reinterpret_cast<float4*>(crow + n) = v;
  } else {
    float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int nn = n + u;
      if (nn >= d.Cout) break;
      float x = e[u];
      if (d.row_scale) x *= d.row_scale[m % d.row_period];
      x = fmaf(x, d.scale ? d.scale[nn] : 1.0f, d.shift ? d.shift[nn] : 0.0f);
      if (d.res1) x += d.res1[m * d.ldr1 + nn];
      x = act_apply(x, d.act);
      if (d.res2) x += d.res2[m * d.ldr2 + nn];
      crow[nn] = x;
    }
  }
}

__device__ __forceinline__ int swz(int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & 7)) << 2); }


template <int TM, int TN, int DB>
__global__ __launch_bounds__(256) void conv_gemm_kernel(const ConvArgs p) {
  constexpr int BM = 64 * TM;
  constexpr int BN = 64 * TN;
  constexpr int PA = BM / 32;  // loader passes (32 rows per pass)
  constexpr int PB = BN / 32;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int EPI = 4 * 32 * (TN * 32);  // epilogue: one 32×(32·TN) slab per wave
  constexpr int SMEM = STAGE * (DB ? 2 : 1) > EPI ? STAGE * (DB ? 2 : 1) : EPI;
  __shared__ __attribute__((aligned(16))) float smem[SMEM];

  const sp_conv_desc& d = p.d;
  const int tid = threadIdx.x;
  const int lrow = tid >> 3;   // 0..31
  const int lchunk = tid & 7;  // 16-byte chunk of the 32-wide k slab
  const int64_t m0 = (int64_t)blockIdx.y * BM;
  const int n0 = blockIdx.x * BN;

  // Per-row implicit-im2col state for this thread's A rows (fixed across k).
  int a_iy0[PA], a_ix0[PA], a_base[PA];
  bool a_ok[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    int64_t m = m0 + i * 32 + lrow;
    a_ok[i] = m < p.M;
    int64_t mm = a_ok[i] ? m : 0;
    int b = (int)(mm / p.HoWo);
    int rem = (int)(mm - (int64_t)b * p.HoWo);
    int oy = rem / d.Wo;
    int ox = rem - oy * d.Wo;
    a_iy0[i] = oy * d.stride - d.pad;
    a_ix0[i] = ox * d.stride - d.pad;
    a_base[i] = b * d.H;
  }

  float4 ra[PA], rb[PB];

  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
    if (p.fast) {
      const int tap = k0 / d.Cin;
      const int c0 = k0 - tap * d.Cin + lchunk * 4;
      const int kh = tap / d.KW;
      const int kw = tap - kh * d.KW;
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const int iy = a_iy0[i] + kh;
        const int ix = a_ix0[i] + kw;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a_ok[i] && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W) {
          const int64_t pix = (int64_t)(a_base[i] + iy) * d.W + ix;
          v = *reinterpret_cast<const float4*>(d.A + pix * d.lda + c0);
          if (d.A2) {
            float4 w = *reinterpret_cast<const float4*>(d.A2 + pix * d.lda2 + c0);
            v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
          }
        }
        ra[i] = v;
      }
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        const int n = n0 + i * 32 + lrow;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (n < d.Cout) v = *reinterpret_cast<const float4*>(d.Wt + (int64_t)n * p.K + k0 + lchunk * 4);
        rb[i] = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        float e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = k0 + lchunk * 4 + j;
          float v = 0.f;
          if (a_ok[i] && k < p.K) {
            const int tap = k / d.Cin;
            const int c = k - tap * d.Cin;
            const int kh = tap / d.KW;
            const int kw = tap - kh * d.KW;
            const int iy = a_iy0[i] + kh;
            const int ix = a_ix0[i] + kw;
            if ((unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W) {
              const int64_t pix = (int64_t)(a_base[i] + iy) * d.W + ix;
              v = d.A[pix * d.lda + c];
              if (d.A2) v += d.A2[pix * d.lda2 + c];
            }
          }
          e[j] = v;
        }
        ra[i] = make_float4(e[0], e[1], e[2], e[3]);
      }
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        const int n = n0 + i * 32 + lrow;
        float e[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = k0 + lchunk * 4 + j;
          e[j] = (n < d.Cout && k < p.K) ? d.Wt[(int64_t)n * p.K + k] : 0.f;
        }
        rb[i] = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
  };

  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int wm = wave >> 1;
  const int wn = wave & 1;
  const int r = lane & 31;
  const int h = lane >> 5;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  const int nk_all = (p.K + BK - 1) / BK;
  const int kt0 = (int)(((int64_t)nk_all * blockIdx.z) / p.splits);
  const int kt1 = (int)(((int64_t)nk_all * (blockIdx.z + 1)) / p.splits);
  const int nk = kt1 - kt0;

  auto store_tile = [&](float* st) {
    float* As = st;
    float* Bs = st + BM * BK;
#pragma unroll
    for (int i = 0; i < PA; ++i)
      *reinterpret_cast<float4*>(As + swz(i * 32 + lrow, lchunk)) = ra[i];
#pragma unroll
    for (int i = 0; i < PB; ++i)
      *reinterpret_cast<float4*>(Bs + swz(i * 32 + lrow, lchunk)) = rb[i];
  };

  auto compute_tile = [&](const float* st) {
    const float* As = st;
    const float* Bs = st + BM * BK;
#pragma unroll
    for (int s = 0; s < BK / 8; ++s) {
      float4 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const float4*>(As + swz(wm * TM * 32 + i * 32 + r, s * 2 + h));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const float4*>(Bs + swz(wn * TN * 32 + j * 32 + r, s * 2 + h));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].x, fb[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].y, fb[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].z, fb[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i].w, fb[j].w, acc[i][j], 0, 0, 0);
        }
    }
  };

  if (nk > 0) load_tile(kt0);
  if (DB && nk > 0) {
    // two LDS stages, one barrier per k-tile: tile t+1's global loads and LDS
    // store overlap tile t's MFMAs.
    store_tile(smem);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) load_tile(kt0 + kt + 1);
      compute_tile(smem + (kt & 1) * STAGE);
      if (kt + 1 < nk) store_tile(smem + ((kt + 1) & 1) * STAGE);
      __syncthreads();
    }
  } else if (!DB) {
    for (int kt = 0; kt < nk; ++kt) {
      __syncthreads();
      store_tile(smem);
      __syncthreads();
      if (kt + 1 < nk) load_tile(kt0 + kt + 1);
      compute_tile(smem);
    }
  }

  // Epilogue, staged through LDS so every lane applies it to a contiguous float4
  // of one output row (16-byte loads of res1/res2/scale/shift, 16-byte stores):
  // pass i moves each wave's 32-row band acc[i][*] to its private LDS slab.
  constexpr int WN = TN * 32;  // columns per wave; LDS rows of WN floats (one bank row at TN=2)
  float* slab = smem + wave * (32 * WN);
  const int nb = n0 + wn * WN;
  __syncthreads();  // main loop done with the operand stages
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q)
        slab[((q & 3) + 8 * (q >> 2) + 4 * h) * WN + j * 32 + r] = acc[i][j][q];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes done
    __builtin_amdgcn_wave_barrier();
    const int64_t mb = m0 + wm * TM * 32 + i * 32;
#pragma unroll
    for (int t = 0; t < (32 * WN / 4) / 64; ++t) {
      const int c = lane + 64 * t;
      const int row = c / (WN / 4);
      const int col = (c - row * (WN / 4)) * 4;
      const int64_t m = mb + row;
      const int n = nb + col;
      if (m >= p.M || n >= d.Cout) continue;
      float4 v = *reinterpret_cast<const float4*>(slab + row * WN + col);
      if (p.splits > 1) {
        *reinterpret_cast<float4*>(p.partial + ((int64_t)blockIdx.z * p.M + m) * p.ldp + n) = v;
      } else {
        epilogue_store(p, m, n, v);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}


// ---------------------------------------------------------------------------------------------
// bf16 variant (SP_PREC_BF16): the same implicit GEMM on v_mfma_f32_32x32x16_bf16 (16× the fp32
// MFMA rate, fp32 accumulate). Activations stay fp32 in HBM and are rounded to bf16 (RNE,
// v_cvt_pk_bf16_f32) while staging into LDS; weights are pre-rounded bf16 [Cout][K]. Tile
// BM×BN×64, two LDS stages (one barrier per k-tile), LDS rows of 64 bf16 = 128 B with the
// same 16-byte-chunk XOR swizzle as the fp32 kernel; lane (r, h) of k-step s reads chunk 2s+h,
// i.e. A[r][16s + 8h + j] — exactly the 32x32x16 operand map.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int BK16 = 64;

__device__ __forceinline__ int swz16(int row, int chunk) { return row * 8 + (chunk ^ ((row >> 1) & 7)); }

template <int TM, int TN>
__global__ __launch_bounds__(256) void conv_gemm_bf16_kernel(const ConvArgs p) {
  constexpr int BM = 64 * TM;
  constexpr int BN = 64 * TN;
  constexpr int PA = BM / 32;
  constexpr int PB = BN / 32;
  constexpr int STAGE = (BM + BN) * 8;           // uint4 per LDS stage
  constexpr int EPI = 4 * 32 * (TN * 32) / 4;    // epilogue slabs in uint4
  constexpr int SMEM = 2 * STAGE > EPI ? 2 * STAGE : EPI;
  __shared__ uint4 smem4[SMEM];
  float* smem = reinterpret_cast<float*>(smem4);

  const sp_conv_desc& d = p.d;
  const uint16_t* Wt16 = d.Wt_bf16;
  const int tid = threadIdx.x;
  const int lrow = tid >> 3;
  const int lchunk = tid & 7;  // 8-k chunk of the 64-wide slab
  const int64_t m0 = (int64_t)blockIdx.y * BM;
  const int n0 = blockIdx.x * BN;

  int a_iy0[PA], a_ix0[PA], a_base[PA];
  bool a_ok[PA];
#pragma unroll
  for (int i = 0; i < PA; ++i) {
    int64_t m = m0 + i * 32 + lrow;
    a_ok[i] = m < p.M;
    int64_t mm = a_ok[i] ? m : 0;
    int b = (int)(mm / p.HoWo);
    int rem = (int)(mm - (int64_t)b * p.HoWo);
    int oy = rem / d.Wo;
    int ox = rem - oy * d.Wo;
    a_iy0[i] = oy * d.stride - d.pad;
    a_ix0[i] = ox * d.stride - d.pad;
    a_base[i] = b * d.H;
  }

  float4 ra[PA][2];
  uint4 rb[PB];

  auto load_tile = [&](int kt) {
    const int k = kt * BK16 + lchunk * 8;
    if (p.fast) {  // Cin % 8 == 0: a chunk of 8 k never straddles a tap
      const int tap = k / d.Cin;
      const int c = k - tap * d.Cin;
      const int kh = tap / d.KW;
      const int kw = tap - kh * d.KW;
      const bool kin = k < p.K;
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        const int iy = a_iy0[i] + kh;
        const int ix = a_ix0[i] + kw;
        float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
        if (kin && a_ok[i] && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W) {
          const float* src = d.A + ((int64_t)(a_base[i] + iy) * d.W + ix) * d.lda + c;
          v0 = *reinterpret_cast<const float4*>(src);
          v1 = *reinterpret_cast<const float4*>(src + 4);
          if (d.A2) {
            const float* s2 = d.A2 + ((int64_t)(a_base[i] + iy) * d.W + ix) * d.lda2 + c;
            float4 w0 = *reinterpret_cast<const float4*>(s2), w1 = *reinterpret_cast<const float4*>(s2 + 4);
            v0.x += w0.x; v0.y += w0.y; v0.z += w0.z; v0.w += w0.w;
            v1.x += w1.x; v1.y += w1.y; v1.z += w1.z; v1.w += w1.w;
          }
        }
        ra[i][0] = v0;
        ra[i][1] = v1;
      }
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        const int n = n0 + i * 32 + lrow;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (kin && n < d.Cout) v = *reinterpret_cast<const uint4*>(Wt16 + (int64_t)n * p.K + k);
        rb[i] = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < PA; ++i) {
        float e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int kk = k + j;
          float v = 0.f;
          if (a_ok[i] && kk < p.K) {
            const int tap = kk / d.Cin;
            const int c = kk - tap * d.Cin;
            const int kh = tap / d.KW;
            const int kw = tap - kh * d.KW;
            const int iy = a_iy0[i] + kh;
            const int ix = a_ix0[i] + kw;
            if ((unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W) {
              const int64_t pix = (int64_t)(a_base[i] + iy) * d.W + ix;
              v = d.A[pix * d.lda + c];
              if (d.A2) v += d.A2[pix * d.lda2 + c];
            }
          }
          e[j] = v;
        }
        ra[i][0] = make_float4(e[0], e[1], e[2], e[3]);
        ra[i][1] = make_float4(e[4], e[5], e[6], e[7]);
      }
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        const int n = n0 + i * 32 + lrow;
        uint16_t e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) e[j] = (n < d.Cout && k + j < p.K) ? Wt16[(int64_t)n * p.K + k + j] : 0;
        rb[i] = make_uint4(e[0] | (uint32_t)e[1] << 16, e[2] | (uint32_t)e[3] << 16, e[4] | (uint32_t)e[5] << 16,
                           e[6] | (uint32_t)e[7] << 16);
      }
    }
  };

  auto store_tile = [&](uint4* st) {
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      bf16x8 v;
      v[0] = (__bf16)ra[i][0].x; v[1] = (__bf16)ra[i][0].y; v[2] = (__bf16)ra[i][0].z; v[3] = (__bf16)ra[i][0].w;
      v[4] = (__bf16)ra[i][1].x; v[5] = (__bf16)ra[i][1].y; v[6] = (__bf16)ra[i][1].z; v[7] = (__bf16)ra[i][1].w;
      *reinterpret_cast<bf16x8*>(st + swz16(i * 32 + lrow, lchunk)) = v;
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) st[BM * 8 + swz16(i * 32 + lrow, lchunk)] = rb[i];
  };

  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int wm = wave >> 1;
  const int wn = wave & 1;
  const int r = lane & 31;
  const int h = lane >> 5;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  auto compute_tile = [&](const uint4* st) {
#pragma unroll
    for (int s = 0; s < BK16 / 16; ++s) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(st + swz16(wm * TM * 32 + i * 32 + r, 2 * s + h));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(st + BM * 8 + swz16(wn * TN * 32 + j * 32 + r, 2 * s + h));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  };

  const int nk_all = (p.K + BK16 - 1) / BK16;
  const int kt0 = (int)(((int64_t)nk_all * blockIdx.z) / p.splits);
  const int kt1 = (int)(((int64_t)nk_all * (blockIdx.z + 1)) / p.splits);
  const int nk = kt1 - kt0;
  if (nk > 0) {
    load_tile(kt0);
    store_tile(smem4);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load_tile(kt0 + kt + 1);
    compute_tile(smem4 + (kt & 1) * STAGE);
    if (kt + 1 < nk) store_tile(smem4 + ((kt + 1) & 1) * STAGE);
    __syncthreads();
  }

  // epilogue: identical accumulator layout to the fp32 kernel
  constexpr int WN = TN * 32;
  float* slab = smem + wave * (32 * WN);
  const int nb = n0 + wn * WN;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q)
        slab[((q & 3) + 8 * (q >> 2) + 4 * h) * WN + j * 32 + r] = acc[i][j][q];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    const int64_t mb = m0 + wm * TM * 32 + i * 32;
#pragma unroll
    for (int t = 0; t < (32 * WN / 4) / 64; ++t) {
      const int c = lane + 64 * t;
      const int row = c / (WN / 4);
      const int col = (c - row * (WN / 4)) * 4;
      const int64_t m = mb + row;
      const int n = nb + col;
      if (m >= p.M || n >= d.Cout) continue;
      float4 v = *reinterpret_cast<const float4*>(slab + row * WN + col);
      if (p.splits > 1) {
        *reinterpret_cast<float4*>(p.partial + ((int64_t)blockIdx.z * p.M + m) * p.ldp + n) = v;
      } else {
        epilogue_store(p, m, n, v);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// Split-K combine: out = epilogue(Σ_z partial[z]) in fixed z order (deterministic).
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const ConvArgs p) {
  const int n4 = (p.d.Cout + 3) / 4;
  const int64_t total = p.M * n4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / n4;
    const int n = (int)(i - m * n4) * 4;
    float4 v = *reinterpret_cast<const float4*>(p.partial + m * p.ldp + n);
    for (int z = 1; z < p.splits; ++z) {
      float4 u = *reinterpret_cast<const float4*>(p.partial + ((int64_t)z * p.M + m) * p.ldp + n);
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    epilogue_store(p, m, n, v);
  }
}

template <int TM, int TN, int DB>
int launch(const ConvArgs& a, hipStream_t s) {
  constexpr int BM = 64 * TM, BN = 64 * TN;
  dim3 grid((a.d.Cout + BN - 1) / BN, (unsigned)((a.M + BM - 1) / BM), a.splits);
  if (a.d.precision == SP_PREC_BF16)
    hipLaunchKernelGGL((conv_gemm_bf16_kernel<TM, TN>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((conv_gemm_kernel<TM, TN, DB>), grid, dim3(256), 0, s, a);
  int rc = check_launch("sp_conv2d");
  if (rc || a.splits == 1) return rc;
  int64_t work = a.M * ((a.d.Cout + 3) / 4);
  int64_t g = (work + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)g), dim3(256), 0, s, a);
  return check_launch("sp_conv2d(split-K reduce)");
}

// Tile override for tuning: SP_CONV_CFG = "<TM><TN><DB>", e.g. "221".
int forced_cfg() {
  const char* e = getenv("SP_CONV_CFG");
  return e ? atoi(e) : -1;
}

}  // namespace
}  // namespace sp

extern "C" int sp_conv2d(const sp_conv_desc* d, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(d != nullptr, "sp_conv2d: null descriptor");
  SP_ARG_CHECK(d->A && d->Wt && d->C, "sp_conv2d: null A/W/C");
  SP_ARG_CHECK(d->N > 0 && d->H > 0 && d->W > 0 && d->Cin > 0 && d->Cout > 0,
               "sp_conv2d: bad shape N=%d H=%d W=%d Cin=%d Cout=%d", d->N, d->H, d->W, d->Cin,
               d->Cout);
  SP_ARG_CHECK(d->KH > 0 && d->KW > 0 && d->stride > 0 && d->pad >= 0, "sp_conv2d: bad kernel");
  const int ho = (d->H + 2 * d->pad - d->KH) / d->stride + 1;
  const int wo = (d->W + 2 * d->pad - d->KW) / d->stride + 1;
  SP_ARG_CHECK(ho == d->Ho && wo == d->Wo, "sp_conv2d: Ho/Wo %dx%d != expected %dx%d", d->Ho,
               d->Wo, ho, wo);
  SP_ARG_CHECK(d->lda >= d->Cin, "sp_conv2d: lda %lld < Cin %d", (long long)d->lda, d->Cin);
  SP_ARG_CHECK(d->act >= 0 && d->act <= 3, "sp_conv2d: bad act %d", d->act);
  SP_ARG_CHECK(!d->row_scale || d->row_period > 0, "sp_conv2d: row_period");
  SP_ARG_CHECK(d->precision == SP_PREC_FP32 || d->precision == SP_PREC_BF16, "sp_conv2d: precision");
  SP_ARG_CHECK(d->precision != SP_PREC_BF16 || d->Wt_bf16, "sp_conv2d: bf16 precision needs Wt_bf16");
  const bool bf = d->precision == SP_PREC_BF16;
  ConvArgs a;
  a.d = *d;
  a.M = (int64_t)d->N * ho * wo;
  a.K = d->KH * d->KW * d->Cin;
  a.HoWo = ho * wo;
  a.fast = (d->Cin % (bf ? 8 : BK) == 0) ? 1 : 0;
  if (a.fast && bf) {
    const bool al = (d->lda % 4 == 0) && ((reinterpret_cast<uintptr_t>(d->A) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(d->Wt_bf16) & 15) == 0) &&
                    (!d->A2 || ((d->lda2 % 4 == 0) && ((reinterpret_cast<uintptr_t>(d->A2) & 15) == 0)));
    if (!al) a.fast = 0;
  } else if (a.fast) {
    // float4 loads: 16-byte aligned rows and bases
    const bool al = (d->lda % 4 == 0) && ((reinterpret_cast<uintptr_t>(d->A) & 15) == 0) &&
                    ((reinterpret_cast<uintptr_t>(d->Wt) & 15) == 0) &&
                    (!d->A2 || ((d->lda2 % 4 == 0) && ((reinterpret_cast<uintptr_t>(d->A2) & 15) == 0)));
    if (!al) a.fast = 0;
  }
  {
    auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    bool v = (d->ldc % 4 == 0) && al16(d->C) && (d->Cout % 4 == 0);
    v = v && (!d->res1 || (d->ldr1 % 4 == 0 && al16(d->res1)));
    v = v && (!d->res2 || (d->ldr2 % 4 == 0 && al16(d->res2)));
    v = v && (!d->scale || al16(d->scale)) && (!d->shift || al16(d->shift));
    v = v && (d->out_rows_per_group == 0 || d->out_group_stride % 4 == 0);
    a.vec_epi = v ? 1 : 0;
  }
  // Split-K when the output tile grid cannot fill the chip (small batches: the /detect bs1
  // path) and the K loop is long: partial sums go to the caller's workspace.
  a.splits = 1;
  a.ldp = (d->Cout + 3) & ~3;
  a.partial = d->workspace;
  {
    const int64_t blocks64 = ((a.M + 63) / 64) * ((d->Cout + 63) / 64);
    const int nk = (a.K + (bf ? BK16 : BK) - 1) / (bf ? BK16 : BK);
    if (d->workspace && blocks64 < 256 && nk >= 16) {
      int sp = (int)((512 + blocks64 - 1) / blocks64);
      if (sp > nk / 8) sp = nk / 8;
      if (sp > 16) sp = 16;
      while (sp > 1 && (int64_t)sp * a.M * a.ldp > d->workspace_elems) --sp;
      if (sp > 1) a.splits = sp;
    }
  }
  hipStream_t s = as_stream(stream);
  if (a.splits > 1) return launch<1, 1, 0>(a, s);
  if (bf) {
    switch (forced_cfg()) {
      case 220: return launch<2, 2, 0>(a, s);
      case 120: return launch<1, 2, 0>(a, s);
      case 110: return launch<1, 1, 0>(a, s);
      default: break;
    }
    const int64_t t128 = ((a.M + 127) / 128) * ((d->Cout + 127) / 128);
    if (d->Cout > 64 && t128 >= 512) return launch<2, 2, 0>(a, s);
    if (d->Cout > 64 && t128 >= 128) return launch<1, 2, 0>(a, s);
    return launch<1, 1, 0>(a, s);
  }
  switch (forced_cfg()) {
    case 220: return launch<2, 2, 0>(a, s);
    case 221: return launch<2, 2, 1>(a, s);
    case 210: return launch<2, 1, 0>(a, s);
    case 211: return launch<2, 1, 1>(a, s);
    case 120: return launch<1, 2, 0>(a, s);
    case 121: return launch<1, 2, 1>(a, s);
    case 110: return launch<1, 1, 0>(a, s);
    case 111: return launch<1, 1, 1>(a, s);
    default: break;
  }
  // Tile choice (measured on MI355X, tools/conv_bench.py): the kernel is latency-bound, so
  // occupancy beats operand reuse except for long-K, wide-N, tall-M convs.
  const int64_t tiles64 = ((a.M + 63) / 64) * ((d->Cout + 63) / 64);
  if (a.K >= 3000 && d->Cout >= 384 && a.M >= 100000) return launch<2, 2, 0>(a, s);
  if (a.K <= 128 || d->Cout <= 64 || tiles64 < 3000) return launch<1, 1, 0>(a, s);
  return launch<1, 2, 0>(a, s);
}
