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
#include "conv_common.h"
#include "tile_table.h"

#ifndef SP_DIAG_KERNELS
#define SP_DIAG_KERNELS 0
#endif

bool sp::conv_gemm_has_fused_ln() { return SP_DIAG_KERNELS != 0; }

namespace sp {

namespace {

constexpr int BK = 32;
// Split-K target for long-K GEMMs on mid-size grids (bs1 /detect path: the CCFM 3×3 at M = 6400 ran
// 300 workgroups × 108 k-tiles; split 2 takes it from 213 to 143 µs).
#ifndef SP_SPLITK_BLOCKS
#define SP_SPLITK_BLOCKS 1024
#endif

__device__ __forceinline__ int swz(int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & 7)) << 2); }


// WM × WN waves (WM·WN = 4), each a (32·TM) × (32·TN) patch: 2×2 is the square default, 4×1 gives
// the 32- and 64-wide N tiles that thin outputs (Cout = 32 / 64: stem, stage 1) need without idle MFMAs.
// CNT: the split-K launches, which may combine in the launch (splitk_combine); every other instance keeps the
// plain epilogue.
template <int TM, int TN, int DB, int WM = 2, bool LN = false, bool CNT = false>
__global__ __launch_bounds__(256) void conv_gemm_kernel(const ConvArgs p) {
  constexpr int WN = 4 / WM;
  static_assert(WM * WN == 4, "four waves per workgroup");
  constexpr int BM = 32 * WM * TM;
  constexpr int BN = 32 * WN * TN;
  constexpr int PA = BM / 32;  // loader passes (32 rows per pass)
  constexpr int PB = BN / 32;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int EPI = LN ? 32 * (BN + 4) : 4 * 32 * (TN * 32);  // epilogue: one 32×(32·TN) slab per wave,
                                                                 // or the 32 whole rows of a LayerNorm tile
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
          SP_BCHECK(pix, (int64_t)d.N * d.H * d.W);
          SP_BCHECK(c0 + 3, d.Cin);
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
        if (n < d.Cout) SP_BCHECK(k0 + lchunk * 4 + 3, p.K);
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
  const int wm = wave / WN;
  const int wn = wave % WN;
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
  __syncthreads();  // main loop done with the operand stages
  if constexpr (LN) {
    static_assert(WM == 1 && TM == 1, "row LayerNorm tiles are 32 rows × the whole N");
    epilogue_rowln<TN>(p, smem, acc[0], m0, wave, lane);
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
    epilogue_band<TN, false, CNT>(p, smem + wave * (32 * TN * 32), acc[i], m0 + wm * TM * 32 + i * 32,
                                  n0 + wn * TN * 32, lane);
  if constexpr (CNT) {
    if (p.counters)  // split-K, combined in this launch by the tile's last workgroup
      splitk_combine<256, BM, BN>(p, reinterpret_cast<int*>(smem), blockIdx.y * gridDim.x + blockIdx.x, m0, n0);
  }
}

// Split-K combine: out = epilogue(Σ_z partial[z]) in fixed z order (deterministic).
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const ConvArgs p) {
  const int n4 = (p.d.Cout + 3) / 4;
  const int64_t total = p.M * n4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / n4;
    const int n = (int)(i - m * n4) * 4;
    SP_BCHECK(((int64_t)(p.splits - 1) * p.M + m) * p.ldp + n + 3, p.d.workspace_elems);
    float4 v = *reinterpret_cast<const float4*>(p.partial + m * p.ldp + n);
    for (int z = 1; z < p.splits; ++z) {
      float4 u = *reinterpret_cast<const float4*>(p.partial + ((int64_t)z * p.M + m) * p.ldp + n);
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    epilogue_store(p, m, n, v);
  }
}

template <int TM, int TN, int DB, int WM = 2, bool LN = false, bool CNT = false>
int launch(const ConvArgs& a, hipStream_t s) {
  constexpr int BM = 32 * WM * TM, BN = 32 * (4 / WM) * TN;
  dim3 grid((a.d.Cout + BN - 1) / BN, (unsigned)((a.M + BM - 1) / BM), a.splits);
  ConvArgs b = a;
  b.counters = CNT ? splitk_counters_for(a, (int64_t)grid.x * grid.y) : nullptr;
  hipLaunchKernelGGL((conv_gemm_kernel<TM, TN, DB, WM, LN, CNT>), grid, dim3(256), 0, s, b);
  int rc = check_launch("sp_conv2d");
  if (rc || a.splits == 1 || b.counters) return rc;
  return launch_splitk_reduce(a, s);
}

// Tile override for tests and tuning tools, set explicitly per thread by sp_set_conv_config (never
// from the environment): "<TM><TN><DB>" for the fp32 kernel (e.g. 221) or the conv_mfma16 config
// number (bf16 / split kernels); -1 = by shape (the production choice).
thread_local int g_forced_cfg = -1;
// bs1 tuning hooks (sp_set_splitk_config): the tile of split-K launches, the split-factor cap and the fewest
// k-tiles that split
thread_local int g_forced_splitk_cfg = -1;
thread_local int g_splitk_max = 16;
thread_local int g_splitk_min_nk = 8;

}  // namespace

int forced_cfg() { return g_forced_cfg; }

int launch_splitk_reduce(const ConvArgs& a, hipStream_t s) {
  int64_t work = a.M * ((a.d.Cout + 3) / 4);
  int64_t g = (work + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)g), dim3(256), 0, s, a);
  return check_launch("sp_conv2d(split-K reduce)");
}

}  // namespace sp

extern "C" int sp_set_conv_config(int cfg) {
  sp::g_forced_cfg = cfg < 0 ? -1 : cfg;
  return 0;
}

extern "C" int sp_set_splitk_config(int cfg, int max_splits, int min_ktiles) {
  sp::g_forced_splitk_cfg = cfg < 0 ? -1 : cfg;
  sp::g_splitk_max = max_splits < 1 ? 16 : (max_splits > 16 ? 16 : max_splits);
  sp::g_splitk_min_nk = min_ktiles < 1 ? 8 : min_ktiles;
  return 0;
}

extern "C" int sp_conv2d(const sp_conv_desc* d, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(d != nullptr, "sp_conv2d: null descriptor");
  SP_ARG_CHECK((d->A || d->A_bf16) && d->Wt && (d->C || d->C_bf16), "sp_conv2d: null A/W/C");
  SP_ARG_CHECK(!(d->res1 && d->res1_bf16) && !(d->res2 && d->res2_bf16) &&
                   !(d->ln_gamma && (d->C_bf16 || d->res1_bf16 || d->res2_bf16)),
               "sp_conv2d: res1 and res1_bf16 together, or bf16 rows with the fused LayerNorm");
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
  SP_ARG_CHECK(d->precision == SP_PREC_FP32 || d->precision == SP_PREC_BF16 ||
                   d->precision == SP_PREC_F32X3,
               "sp_conv2d: precision %d", d->precision);
  const int planes = d->precision == SP_PREC_BF16 ? 1 : d->precision == SP_PREC_F32X3 ? 3 : 0;
  SP_ARG_CHECK(!(d->C_bf16 || d->res1_bf16 || d->res2_bf16) || planes == 1,
               "sp_conv2d: bf16 output / residual rows need the bf16 operand mode (SP_PREC_BF16)");
  SP_ARG_CHECK(planes == 0 || d->Wt_bf16, "sp_conv2d: bf16 / split precision needs Wt_bf16");
  const int64_t K = (int64_t)d->KH * d->KW * d->Cin;
  SP_ARG_CHECK(planes < 3 || d->wt_plane_stride >= (int64_t)d->Cout * K,
               "sp_conv2d: wt_plane_stride %lld < Cout*K", (long long)d->wt_plane_stride);
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (d->A_bf16) {
    SP_ARG_CHECK(planes == 1 && !d->A2 && !d->ln_gamma && d->Cin % BK == 0 && d->lda % 8 == 0 && al16(d->A_bf16),
                 "sp_conv2d: bf16 A rows need the bf16 operand mode, Cin %% 32 == 0, lda %% 8 == 0, 16-byte "
                 "alignment, no A2 / LayerNorm");
  }
  ConvArgs a;
  a.d = *d;
  a.A16 = d->A_bf16;
  a.M = (int64_t)d->N * ho * wo;
  a.K = (int32_t)K;
  a.HoWo = ho * wo;
  // fast operand path: every 32-deep k-tile lies in one filter tap, and the rows loaded as
  // float4 / 8 x bf16 are 16-byte aligned.
  a.fast = (d->Cin % BK == 0) ? 1 : 0;
  if (a.fast) {
    bool al = d->A_bf16 || ((d->lda % 4 == 0) && al16(d->A) && (!d->A2 || ((d->lda2 % 4 == 0) && al16(d->A2))));
    al = al && (planes ? (al16(d->Wt_bf16) && (planes == 1 || d->wt_plane_stride % 8 == 0)) : al16(d->Wt));
    if (!al) a.fast = 0;
  }
  {
    auto al8 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 7) == 0; };
    bool v = (d->ldc % 4 == 0) && (d->C_bf16 ? al8(d->C_bf16) : al16(d->C)) && (d->Cout % 4 == 0);
    v = v && (!d->res1 || (d->ldr1 % 4 == 0 && al16(d->res1)));
    v = v && (!d->res1_bf16 || (d->ldr1 % 4 == 0 && al8(d->res1_bf16)));
    v = v && (!d->res2_bf16 || (d->ldr2 % 4 == 0 && al8(d->res2_bf16)));
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
    const int nk = (a.K + BK - 1) / BK;
    // measured at bs1 (profiles/r1/bs1_detail_*.json): short grids split to ~512 workgroups with
    // ≥ 8 k-tiles each; tiny-M linears (< 64 tiles) split even at K = 256; grids of up to
    // SP_SPLITK_BLOCKS tiles split only when each workgroup would walk ≥ 64 k-tiles.
    int sp = 1;
    if (nk < g_splitk_min_nk) sp = 1;
    else if (blocks64 < 64 && nk >= 8 && nk < 16) sp = nk / 4;
    else if (blocks64 < 256 && nk >= 16) sp = (int)((512 + blocks64 - 1) / blocks64), sp = sp < nk / 8 ? sp : nk / 8;
    else if (blocks64 < SP_SPLITK_BLOCKS && nk >= 64) sp = (int)((SP_SPLITK_BLOCKS + blocks64 - 1) / blocks64);
    // split-K runs on the register-staged tiles (fp32 A) and reduces through the fp32-row epilogue
    if (d->workspace && sp > 1 && !d->A_bf16 && !d->C_bf16 && !d->res1_bf16 && !d->res2_bf16) {
      if (sp > g_splitk_max) sp = g_splitk_max;
      while (sp > 1 && (int64_t)sp * a.M * a.ldp > d->workspace_elems) --sp;
      if (sp > 1) a.splits = sp;
    }
  }
  hipStream_t s = as_stream(stream);
  if (d->ln_gamma) {  // Linear → +residual → LayerNorm in one launch: 32-row tiles holding whole rows
    SP_ARG_CHECK(planes == 0 && d->Cout % 128 == 0 && d->Cout <= 512 && d->act == SP_ACT_NONE && !d->res2 &&
                     d->out_rows_per_group == 0 && d->ln_beta && a.fast,
                 "sp_conv2d: fused LayerNorm needs fp32 weights, Cout %% 128 == 0 <= 512, no act / res2 / "
                 "grouped rows, Cin %% 32 == 0 (Cout=%d)", d->Cout);
    a.splits = 1;
#if SP_DIAG_KERNELS
    switch (d->Cout / 128) {
      case 1: return launch<1, 1, 1, 1, true>(a, s);
      case 2: return launch<1, 2, 1, 1, true>(a, s);
      case 3: return launch<1, 3, 1, 1, true>(a, s);
      default: return launch<1, 4, 1, 1, true>(a, s);
    }
#else
    // measured slower than the unfused LayerNorm (58.1 vs 56.7 ms per step) and off by default:
    // the fused-LN tiles are compiled into diagnostic builds only (UNIT=conv_gemm tools/build_diag.sh ...
    // -DSP_DIAG_KERNELS=1)
    set_error("sp_conv2d: the fused LayerNorm epilogue (ln_gamma) is in the diagnostic build only");
    return -1;
#endif
  }
  // tile choice: a test / tuning override, else the measured exact-shape table (tile_table.h),
  // else the by-shape rules below and in launch_mfma16
  int cfg = forced_cfg();
  if (cfg < 0 && a.splits == 1)
    cfg = tile_table_lookup(a.M, d->Cout, a.K, d->KH, d->stride, planes);
  if (cfg < 0 && a.splits > 1 && planes && g_forced_splitk_cfg >= 0) cfg = g_forced_splitk_cfg;
  if (planes) return launch_mfma16(a, planes, cfg, s);
  if (a.splits > 1 && splitk_counters_for(a, ((a.d.Cout + 63) / 64) * ((a.M + 63) / 64)))
    return launch<1, 1, 0, 2, false, true>(a, s);  // the in-launch combine (launch<1, 1, 0>: 64×64 tiles)
  if (a.splits > 1) return launch<1, 1, 0>(a, s);
  switch (cfg) {
    case 220: return launch<2, 2, 0>(a, s);
    case 221: return launch<2, 2, 1>(a, s);
    case 210: return launch<2, 1, 0>(a, s);
    case 211: return launch<2, 1, 1>(a, s);
    case 120: return launch<1, 2, 0>(a, s);
    case 121: return launch<1, 2, 1>(a, s);
    case 110: return launch<1, 1, 0>(a, s);
    case 111: return launch<1, 1, 1>(a, s);
    // 1×4 wave grids: "1<TM><TN><DB>" → tile 32 × (128·TN) (small-M linears: more workgroups)
    case 1110: return launch<1, 1, 0, 1>(a, s);
    case 1111: return launch<1, 1, 1, 1>(a, s);
    case 1120: return launch<1, 2, 0, 1>(a, s);
    case 1121: return launch<1, 2, 1, 1>(a, s);
    // 4×1 wave grids: "4<TM><TN><DB>" → tile (128·TM) × (32·TN)
    case 4110: return launch<1, 1, 0, 4>(a, s);
    case 4111: return launch<1, 1, 1, 4>(a, s);
    case 4210: return launch<2, 1, 0, 4>(a, s);
    case 4211: return launch<2, 1, 1, 4>(a, s);
    case 4120: return launch<1, 2, 0, 4>(a, s);
    case 4121: return launch<1, 2, 1, 4>(a, s);
    default: break;
  }
  // Tile choice (measured on MI355X, tools/conv_bench.py): the kernel is latency-bound, so
  // occupancy beats operand reuse except for long-K, wide-N, tall-M convs.
  const int64_t tiles64 = ((a.M + 63) / 64) * ((d->Cout + 63) / 64);
  // Cout <= 32 (stem): the 4×1 wave grid's 128×32 tile, no idle N half (1.69× on the stem 3×3,
  // 1.23× on the Cin = 3 stem conv; gpurun_out/s5 → profiles/r1/conv_bench_thin_fp32.jsonl).
  if (d->Cout <= 32) return launch<1, 1, 0, 4>(a, s);
  if (d->Cout <= 64 && a.M >= 500000 && a.K >= 288) return launch<2, 1, 0>(a, s);
  if (a.K >= 3000 && d->Cout >= 384 && a.M >= 100000) return launch<2, 2, 0>(a, s);
  if (a.K <= 128 || d->Cout <= 64 || tiles64 < 3000) return launch<1, 1, 0>(a, s);
  return launch<1, 2, 0>(a, s);
}

extern "C" int sp_set_tuning(int knob, int value) {
  switch (knob) {
    case SP_TUNE_GLDS_EPILOGUE:
      sp::set_glds_epilogue(value == 4 ? 4 : -1);
      return 0;
    case SP_TUNE_MSDA_GENERIC:
      sp::set_msda_generic(value == 1 ? 1 : 0);
      return 0;
    default:
      sp::set_error("sp_set_tuning: unknown knob %d", knob);
      return -1;
  }
}
