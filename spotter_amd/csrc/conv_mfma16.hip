// Implicit-GEMM convolution / linear layer on bf16-operand MFMA (v_mfma_f32_32x32x16_bf16,
// fp32 accumulate) for gfx950. Two operand modes share one kernel body:
//
//   PL = 1  bf16: activations rounded RNE to bf16 while staging, weights pre-rounded bf16
//           (sp_precision SP_PREC_BF16, the separately reported bf16 variant);
//   PL = 3  fp32 via a 3-way split (SP_PREC_F32X3): each fp32 operand x = hi + mid + lo with
//           hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid) (both differences are exact
//           in fp32), so the three planes hold all 24 significand bits. Per 16-deep k step the
//           wave issues the six products down to the 2^-17 |a b| scale:
//             lo·hi, hi·lo, mid·mid, mid·hi, hi·mid, hi·hi   (smallest first)
//           With round-to-nearest |mid| <= 2^-8 |x| and |lo| <= 2^-17 |x|, so the dropped mid·lo,
//           lo·mid, lo·lo terms sum to <= 2^-24 |a b| — one fp32 rounding of the product — and
//           every bf16×bf16 product is exact in the fp32 accumulator. The MFMA
//           accumulator is rounded 6 times per 16 k here versus 16 times for the fp32 MFMA
//           (v_mfma_f32_32x32x2_f32 ≡ an fmaf chain), so the result is fp32-accurate while the
//           matrix core runs 6 × 32 = 192 cycles per 32×32×16 block instead of 8 × 64 = 512.
//
// Same GEMM contract and fused epilogue as conv_gemm.hip (conv_common.h): A gathered on the fly
// from NHWC activations (implicit im2col), W as [Cout][K] bf16 planes (k contiguous).
//
// Tiling: WM×WN waves per workgroup, each wave a (32·TM)×(32·TN) patch of 32×32 accumulators;
// BK = 32 k per LDS stage (two 16-deep MFMA steps). Operand tiles are staged global → registers
// (fp32 A split into planes on the way) → LDS, double-buffered with one barrier per k-tile.
// LDS planes are [rows][32 bf16] = four 16-byte chunks per row; chunk c of row r lives at
// r·4 + (c ^ ((r >> 2) & 3)), which makes the 16-lane groups of every ds_read_b128 fragment
// read (lanes r = 0..31 of one chunk) hit 16 distinct bank slots, and keeps the 8-lane groups
// of the ds_write_b128 staging stores conflict-free.
// The 1-D grid is remapped XCD-aware (MI355X dispatches consecutive workgroups round-robin over
// the 8 XCDs): each XCD receives a contiguous run of output tiles, N fastest, so workgroups that
// share an A row-panel share one L2.
#include <cstdlib>

#include <type_traits>

#include "mfma16_common.h"

#ifndef SP_ABLATE
#define SP_ABLATE 0
#endif
// conv_x3s_kernel ablation bits (timing experiments only; results are wrong with any bit set):
// 1 no in-loop DMA, 2 no A split (raw bits), 4 no MFMA, 8 no in-loop barrier
#ifndef SP_X3S_ABL
#define SP_X3S_ABL 0
#endif
// Diagnostic build only (-DSP_X3S_STAMP): s_memtime stamps of the first 64 intervals of every wave of
// workgroup 0 of a conv_x3s_kernel launch, stored by lane 0 with vector stores, read back with
// sp_debug_x3s_stamps (tools/microbench/x3s_stamps.py). Not in the product build.
#ifndef SP_X3S_STAMP
#define SP_X3S_STAMP 0
#endif

namespace sp {

namespace {

// CNT: a split-K instance, which may combine in the launch (splitk_combine); other instances keep the plain
// epilogue.
template <int WM, int WN, int TM, int TN, int PL, bool FAST, bool CNT = false>
__global__ __launch_bounds__(64 * WM * WN) void conv_mfma16_kernel(const ConvArgs p) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BM = 32 * TM * WM;
  constexpr int BN = 32 * TN * WN;
  constexpr int TA = BM * 4 / NT;             // A chunk tasks (8 k each) per thread
  constexpr int TB = (BN * 4 + NT - 1) / NT;  // B chunk tasks per thread (last may be partial)
  constexpr bool BFULL = (BN * 4) % NT == 0;
  static_assert(TA * NT == BM * 4, "A staging must tile the workgroup");
  constexpr int PA = BM * 4;  // uint4 per A plane
  constexpr int PB = BN * 4;  // uint4 per B plane
  constexpr int STAGE = PL * (PA + PB);
  constexpr int NB = (WM * WN * TM * 32 * TN * 32 / 4 <= 2 * STAGE) ? TM : 1;  // epilogue bands per round
  constexpr int EPI = WM * WN * NB * 32 * TN * 32 / 4;
  constexpr int SMEM = 2 * STAGE > EPI ? 2 * STAGE : EPI;
  __shared__ uint4 smem[SMEM];

  const sp_conv_desc& d = p.d;
  const int64_t wps = d.wt_plane_stride;
  const int tid = threadIdx.x;
  const int c = tid & 3;  // this thread's 8-k chunk of every staged row

  // XCD-aware tile order (bijective for any grid size).
  const int tilesN = (d.Cout + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int mt = wg / tilesN;
  const int n0 = (wg - mt * tilesN) * BN;
  const int64_t m0 = (int64_t)mt * BM;

  // Per A task: the im2col row's origin (iy0, ix0) and a pointer to its tap-(0,0) pixel
  // (+ this thread's chunk); rows past M are parked out of bounds (iy0 = -2^20).
  int a_iy0[TA], a_ix0[TA];
  const float* a_ptr[TA];
  const float* a2_ptr[TA];
#pragma unroll
  for (int i = 0; i < TA; ++i) {
    const int64_t m = m0 + ((tid + NT * i) >> 2);
    const bool ok = m < p.M;
    const int64_t mm = ok ? m : 0;
    const int b = (int)(mm / p.HoWo);
    const int rem = (int)(mm - (int64_t)b * p.HoWo);
    const int oy = rem / d.Wo;
    const int ox = rem - oy * d.Wo;
    a_iy0[i] = ok ? oy * d.stride - d.pad : -(1 << 20);
    a_ix0[i] = ox * d.stride - d.pad;
    const int64_t pix = ((int64_t)b * d.H + a_iy0[i]) * d.W + a_ix0[i];
    a_ptr[i] = d.A + pix * d.lda + c * 8;
    a2_ptr[i] = d.A2 ? d.A2 + pix * d.lda2 + c * 8 : nullptr;
  }
  const uint16_t* b_ptr[TB];
#pragma unroll
  for (int i = 0; i < TB; ++i) {
    const int n = n0 + ((tid + NT * i) >> 2);
    b_ptr[i] = d.Wt_bf16 + (int64_t)(n < d.Cout ? n : 0) * p.K + c * 8;
  }

  float4 ra[TA][2];
  uint4 rb[TB][PL];

  // FAST (Cin % 32 == 0): a 32-deep k-tile lies inside one filter tap, so the tap walk is
  // wave-uniform scalar state (kh, kw, c0) advanced once per tile.
  int s_kh = 0, s_kw = 0, s_c0 = 0;
  auto seek = [&](int kt) {
    const int k0 = kt * KT;
    const int tap = k0 / d.Cin;
    s_c0 = k0 - tap * d.Cin;
    s_kh = tap / d.KW;
    s_kw = tap - s_kh * d.KW;
  };

  auto load_tile = [&](int kt) {
    const int k0 = kt * KT;
    if constexpr (FAST) {
      const int64_t off = ((int64_t)s_kh * d.W + s_kw) * d.lda + s_c0;
      const int64_t off2 = ((int64_t)s_kh * d.W + s_kw) * d.lda2 + s_c0;
#pragma unroll
      for (int i = 0; i < TA; ++i) {
        float4 v0 = make_float4(0.f, 0.f, 0.f, 0.f), v1 = v0;
        if ((unsigned)(a_iy0[i] + s_kh) < (unsigned)d.H && (unsigned)(a_ix0[i] + s_kw) < (unsigned)d.W) {
          const float* src = a_ptr[i] + off;
          v0 = *reinterpret_cast<const float4*>(src);
          v1 = *reinterpret_cast<const float4*>(src + 4);
          if (d.A2) {
            const float* s2 = a2_ptr[i] + off2;
            const float4 w0 = *reinterpret_cast<const float4*>(s2);
            const float4 w1 = *reinterpret_cast<const float4*>(s2 + 4);
            v0.x += w0.x; v0.y += w0.y; v0.z += w0.z; v0.w += w0.w;
            v1.x += w1.x; v1.y += w1.y; v1.z += w1.z; v1.w += w1.w;
          }
        }
        ra[i][0] = v0;
        ra[i][1] = v1;
      }
#pragma unroll
      for (int i = 0; i < TB; ++i) {
        const int t = tid + NT * i;
        const bool ok = (BFULL || t < BN * 4) && n0 + (t >> 2) < d.Cout;
#pragma unroll
        for (int pl = 0; pl < PL; ++pl)
          rb[i][pl] = ok ? *reinterpret_cast<const uint4*>(b_ptr[i] + k0 + pl * wps) : make_uint4(0u, 0u, 0u, 0u);
      }
      // advance the tap walk to the next k-tile
      s_c0 += KT;
      if (s_c0 >= d.Cin) {
        s_c0 = 0;
        if (++s_kw == d.KW) {
          s_kw = 0;
          ++s_kh;
        }
      }
    } else {  // generic gather (Cin = 3 stem, K = 4 query-pos head): element-wise, k < K checked
      const int k = k0 + c * 8;
#pragma unroll
      for (int i = 0; i < TA; ++i) {
        float e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int kk = k + j;
          float v = 0.f;
          if (kk < p.K) {
            const int tap = kk / d.Cin;
            const int ch = kk - tap * d.Cin;
            const int kh = tap / d.KW;
            const int kw = tap - kh * d.KW;
            if ((unsigned)(a_iy0[i] + kh) < (unsigned)d.H && (unsigned)(a_ix0[i] + kw) < (unsigned)d.W) {
              const int64_t o = ((int64_t)kh * d.W + kw) * d.lda + ch - c * 8;
              v = a_ptr[i][o];
              if (d.A2) v += a2_ptr[i][((int64_t)kh * d.W + kw) * d.lda2 + ch - c * 8];
            }
          }
          e[j] = v;
        }
        ra[i][0] = make_float4(e[0], e[1], e[2], e[3]);
        ra[i][1] = make_float4(e[4], e[5], e[6], e[7]);
      }
#pragma unroll
      for (int i = 0; i < TB; ++i) {
        const int t = tid + NT * i;
        const bool nok = (BFULL || t < BN * 4) && n0 + (t >> 2) < d.Cout;
#pragma unroll
        for (int pl = 0; pl < PL; ++pl) {
          uint16_t e[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = (nok && k + j < p.K) ? b_ptr[i][k0 + j + pl * wps] : (uint16_t)0;
          rb[i][pl] = make_uint4(e[0] | (uint32_t)e[1] << 16, e[2] | (uint32_t)e[3] << 16,
                                 e[4] | (uint32_t)e[5] << 16, e[6] | (uint32_t)e[7] << 16);
        }
      }
    }
  };

  auto store_tile = [&](uint4* st) {
#pragma unroll
    for (int i = 0; i < TA; ++i) {
      bf16x8 pv[PL];
      split_frag_pk<PL>(ra[i][0], ra[i][1], pv);
      const int row = (tid + NT * i) >> 2;
#pragma unroll
      for (int pl = 0; pl < PL; ++pl) *reinterpret_cast<bf16x8*>(st + pl * PA + sw16(row, c)) = pv[pl];
    }
#pragma unroll
    for (int i = 0; i < TB; ++i) {
      const int t = tid + NT * i;
      if (BFULL || t < BN * 4) {
#pragma unroll
        for (int pl = 0; pl < PL; ++pl) st[PL * PA + pl * PB + sw16(t >> 2, c)] = rb[i][pl];
      }
    }
  };

  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int wm = wave / WN;
  const int wn = wave - wm * WN;
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
    for (int s = 0; s < KT / 16; ++s) {
      bf16x8 fa[TM][PL], fb[TN][PL];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int pl = 0; pl < PL; ++pl)
          fa[i][pl] = *reinterpret_cast<const bf16x8*>(st + pl * PA + sw16(wm * TM * 32 + i * 32 + r, 2 * s + h));
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int pl = 0; pl < PL; ++pl)
          fb[j][pl] = *reinterpret_cast<const bf16x8*>(st + PL * PA + pl * PB +
                                                       sw16(wn * TN * 32 + j * 32 + r, 2 * s + h));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_planes<PL>(fa[i], fb[j], acc[i][j]);
    }
  };

  const int nk_all = (p.K + KT - 1) / KT;
  const int kt0 = (int)(((int64_t)nk_all * blockIdx.z) / p.splits);
  const int kt1 = (int)(((int64_t)nk_all * (blockIdx.z + 1)) / p.splits);
  const int nk = kt1 - kt0;
  if constexpr (FAST) seek(kt0);
  if (nk > 0) {
    load_tile(kt0);
    store_tile(smem);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load_tile(kt0 + kt + 1);
    compute_tile(smem + (kt & 1) * STAGE);
    if (kt + 1 < nk) store_tile(smem + ((kt + 1) & 1) * STAGE);
    __syncthreads();
  }

  float* smemf = reinterpret_cast<float*>(smem);
  epilogue_tile<TM, TN, NB, false, PL == 1, CNT>(p, smemf + wave * (NB * 32 * TN * 32), acc, m0 + wm * TM * 32,
                                                  n0 + wn * TN * 32, lane);
  if constexpr (CNT) {
    if (p.counters)  // split-K, combined in this launch by the tile's last workgroup
      splitk_combine<NT, BM, BN>(p, reinterpret_cast<int*>(smem), wg, m0, n0);
  }
}

#if SP_X3S_STAMP
__device__ unsigned long long g_x3s_stamps[8 * 64 * 8];
#endif

// The software-pipelined (conv_pipe, cfg 21-26) and ping-pong (conv_pp, cfg 31-32) kernels below measured slower
// than the LDS-DMA tiles on every C2 / C3 / C5 shape and are in no tile table: diagnostic builds only
// (UNIT=conv_mfma16 tools/build_diag.sh <name> -DSP_DIAG_KERNELS=1), not the product library.
#ifndef SP_DIAG_KERNELS
#define SP_DIAG_KERNELS 0
#endif
#if SP_DIAG_KERNELS
// ---------------------------------------------------------------------------------------------
// Software-pipelined LDS-DMA variant: as conv_glds_kernel, plus the fragment loads (ds_read +
// bf16 split) of k16 step t+1 are issued between the MFMAs of step t (sched_group_barrier
// interleave), so one wave per SIMD keeps its matrix pipe fed: the split VALU work and the LDS
// read latency hide under the MFMA chain. One raw barrier per k-tile sits between its two k16
// steps: by then every wave has consumed its reads of the buffer being refilled, and stage kt+1
// has been waited for (vmcnt counted; NS-3 stages stay in flight) so the second half can prefetch
// the next tile's first step.
template <int WM, int WN, int TM, int TN, int PL, int NS>
__global__ __launch_bounds__(64 * WM * WN) void conv_pipe_kernel(const ConvArgs p) {
  constexpr int NT = 64 * WM * WN;
  constexpr int BM = 32 * TM * WM;
  constexpr int BN = 32 * TN * WN;
  constexpr int CA = BM * 8;
  constexpr int CB = BN * 4;
  constexpr int GA = CA / NT;
  constexpr int GB = CB / NT;
  static_assert(GA * NT == CA && GB * NT == CB && GB >= 1, "DMA pieces must tile the workgroup");
  constexpr int GLDS = GA + PL * GB;
  constexpr int STAGE = CA + PL * CB;
  constexpr int NB = (WM * WN * TM * 32 * TN * 32 / 4 <= NS * STAGE) ? TM : 1;
  constexpr int EPI = WM * WN * NB * 32 * TN * 32 / 4;
  constexpr int SMEM = NS * STAGE > EPI ? NS * STAGE : EPI;
  static_assert(NS >= 3 && NS <= 4, "stages");
  __shared__ uint4 smem[SMEM];

  const sp_conv_desc& d = p.d;
  const int64_t wps = d.wt_plane_stride;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;

  const int tilesN = (d.Cout + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int mt = wg / tilesN;
  const int n0 = (wg - mt * tilesN) * BN;
  const int64_t m0 = (int64_t)mt * BM;

  const int ca = (tid & 7) ^ (((tid >> 3) >> 1) & 7);
  int a_iy0[GA], a_ix0[GA];
  const float* a_ptr[GA];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int64_t m = m0 + ((j * NT + tid) >> 3);
    const bool ok = m < p.M;
    const int64_t mm = ok ? m : 0;
    const int b = (int)(mm / p.HoWo);
    const int rem = (int)(mm - (int64_t)b * p.HoWo);
    const int oy = rem / d.Wo;
    const int ox = rem - oy * d.Wo;
    a_iy0[j] = ok ? oy * d.stride - d.pad : -(1 << 20);
    a_ix0[j] = ox * d.stride - d.pad;
    a_ptr[j] = d.A + (((int64_t)b * d.H + a_iy0[j]) * d.W + a_ix0[j]) * d.lda + ca * 4;
  }
  const int cbk = (tid & 3) ^ (((tid >> 2) >> 2) & 3);
  const uint16_t* b_ptr[GB];
  bool b_ok[GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int n = n0 + ((j * NT + tid) >> 2);
    b_ok[j] = n < d.Cout;
    b_ptr[j] = d.Wt_bf16 + (int64_t)(b_ok[j] ? n : 0) * p.K + cbk * 8;
  }
  const char* zero = reinterpret_cast<const char*>(g_zero_chunk);

  int s_kh = 0, s_kw = 0, s_c0 = 0;
  const int nk_all = p.K / KT;
  const int kt0 = (int)(((int64_t)nk_all * blockIdx.z) / p.splits);
  const int kt1 = (int)(((int64_t)nk_all * (blockIdx.z + 1)) / p.splits);
  const int nk = kt1 - kt0;
  {
    const int k0 = kt0 * KT;
    const int tap = k0 / d.Cin;
    s_c0 = k0 - tap * d.Cin;
    s_kh = tap / d.KW;
    s_kw = tap - s_kh * d.KW;
  }

  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)smem;
  const uint32_t wave_off = (uint32_t)__builtin_amdgcn_readfirstlane(wave * 64 * 16);
  auto issue = [&](int kt, int buf) {
    const uint32_t st = lds0 + (uint32_t)(buf * STAGE * 16) + wave_off;
    const int64_t off = ((int64_t)s_kh * d.W + s_kw) * d.lda + s_c0;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const bool ok = (unsigned)(a_iy0[j] + s_kh) < (unsigned)d.H && (unsigned)(a_ix0[j] + s_kw) < (unsigned)d.W;
      const void* src = ok ? static_cast<const void*>(a_ptr[j] + off) : static_cast<const void*>(zero + ca * 16);
      glds16(src, st + j * NT * 16);
    }
    const int k0 = kt * KT;
#pragma unroll
    for (int pl = 0; pl < PL; ++pl)
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const void* src = b_ok[j] ? static_cast<const void*>(b_ptr[j] + pl * wps + k0)
                                  : static_cast<const void*>(zero + cbk * 16);
        glds16(src, st + (CA + pl * CB + j * NT) * 16);
      }
    s_c0 += KT;
    if (s_c0 >= d.Cin) {
      s_c0 = 0;
      if (++s_kw == d.KW) {
        s_kw = 0;
        ++s_kh;
      }
    }
  };

  const int wm = wave / WN;
  const int wn = wave - wm * WN;
  const int r = lane & 31;
  const int h = lane >> 5;
  int a_row[TM], a_sz[TM], b_row[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    a_row[i] = (wm * TM * 32 + i * 32 + r) * 8;
    a_sz[i] = ((wm * TM * 32 + i * 32 + r) >> 1) & 7;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) b_row[j] = wn * TN * 32 + j * 32 + r;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  bf16x8 fa0[TM][PL], fb0[TN][PL], fa1[TM][PL], fb1[TN][PL];

  // fragments of k16 step s (0/1) of stage buffer `buf`
  auto frags = [&](int buf, int s, bf16x8 (&fa)[TM][PL], bf16x8 (&fb)[TN][PL]) {
    const uint4* st = smem + buf * STAGE;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int pl = 0; pl < PL; ++pl)
        fb[j][pl] = *reinterpret_cast<const bf16x8*>(st + CA + pl * CB + sw16(b_row[j], 2 * s + h));
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int c0 = 4 * s + 2 * h;
      const float4 x0 = *reinterpret_cast<const float4*>(st + a_row[i] + (c0 ^ a_sz[i]));
      const float4 x1 = *reinterpret_cast<const float4*>(st + a_row[i] + ((c0 + 1) ^ a_sz[i]));
      split_frag_pk<PL>(x0, x1, fa[i]);
    }
  };
  auto mma = [&](const bf16x8 (&fa)[TM][PL], const bf16x8 (&fb)[TN][PL]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma_planes<PL>(fa[i], fb[j], acc[i][j]);
  };
  // per MFMA of the current step: first the next step's ds_reads (2 per gap), then its VALU
  constexpr int NMF = TM * TN * (PL == 3 ? 6 : 1);
  constexpr int NDS = TM * 2 + TN * PL;
  constexpr int NVALU = TM * (PL == 3 ? 48 : 8) + 8;
  constexpr int VSTART = NMF > 4 ? 2 : 1;
  constexpr int VPER = (NVALU + (NMF - VSTART) - 1) / (NMF - VSTART > 0 ? NMF - VSTART : 1);
  auto interleave = [&]() {
#pragma unroll
    for (int i = 0; i < NMF; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (i < (NDS + 1) / 2) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      if (i >= VSTART) __builtin_amdgcn_sched_group_barrier(0x002, VPER, 0);
    }
  };

  // prologue: stages 0 .. NS-2 in flight; stage 0 landed for everyone; step-0 fragments
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(kt0 + t, t);
  if (nk > 0) {
    if (nk >= NS - 1) {
      wait_vmcnt<(NS - 2) * GLDS>();
    } else {
      wait_vmcnt<0>();
    }
    raw_barrier();
    frags(0, 0, fa0, fb0);
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % NS;
    const int nxt = (kt + 1) % NS;
    // half A: MFMAs of step (kt, 0) ‖ fragments of step (kt, 1)
    frags(cur, 1, fa1, fb1);
    mma(fa0, fb0);
    interleave();
    // stage kt+1 landed (stages up to kt+NS-2 issued; NS-3 of them may stay in flight)
    if constexpr (NS == 4) {
      if (kt + 2 < nk) wait_vmcnt<GLDS>();
      else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    raw_barrier();  // every wave is past its reads of buffer (kt-1) % NS → refill it
    if (kt + NS - 1 < nk) issue(kt0 + kt + NS - 1, (kt + NS - 1) % NS);
    // half B: MFMAs of step (kt, 1) ‖ fragments of step (kt+1, 0) (a harmless stale read after the last tile)
    frags(nxt, 0, fa0, fb0);
    mma(fa1, fb1);
    interleave();
  }

  __syncthreads();
  float* smemf = reinterpret_cast<float*>(smem);
  epilogue_tile<TM, TN, NB, false, PL == 1, CNT>(p, smemf + wave * (NB * 32 * TN * 32), acc, m0 + wm * TM * 32,
                                                  n0 + wn * TN * 32, lane);
  if constexpr (CNT) {
    if (p.counters)  // split-K, combined in this launch by the tile's last workgroup
      splitk_combine<NT, BM, BN>(p, reinterpret_cast<int*>(smem), wg, m0, n0);
  }
}

template <int WM, int WN, int TM, int TN, int NS>
int launch_pipe(const ConvArgs& a, int planes, hipStream_t s) {
  constexpr int BM = 32 * TM * WM, BN = 32 * TN * WN;
  const int64_t tiles = ((a.M + BM - 1) / BM) * ((a.d.Cout + BN - 1) / BN);
  if (tiles > 0x7fffffff) {
    set_error("sp_conv2d: %lld tiles exceed the grid", (long long)tiles);
    return -1;
  }
  dim3 grid((unsigned)tiles, 1, a.splits);
  // NS stages of the fp32 A tile + PL bf16 B planes must fit the 160 KiB LDS
  constexpr bool fits3 = NS * (BM * 8 + 3 * BN * 4) * 16 <= 163840;
  if (planes == 3) {
    if constexpr (fits3) {
      hipLaunchKernelGGL((conv_pipe_kernel<WM, WN, TM, TN, 3, NS>), grid, dim3(64 * WM * WN), 0, s, a);
    } else {
      set_error("sp_conv2d: pipe tile %dx%d with %d stages does not fit LDS in f32x3 mode", BM, BN, NS);
      return -1;
    }
  } else {
    hipLaunchKernelGGL((conv_pipe_kernel<WM, WN, TM, TN, 1, NS>), grid, dim3(64 * WM * WN), 0, s, a);
  }
  int rc = check_launch(planes == 3 ? "sp_conv2d(f32x3 pipe)" : "sp_conv2d(bf16 pipe)");
  if (rc || a.splits == 1) return rc;
  return launch_splitk_reduce(a, s);
}

// ---------------------------------------------------------------------------------------------
// Ping-pong LDS-DMA kernel: 8 waves as two groups of four (waves 0-3 = group A, 4-7 = group B; a
// workgroup's waves land on the 4 SIMDs in turn, so every SIMD holds one wave of each group). Per
// k-tile a wave runs a MEMORY phase (fragment ds_reads + the fp32→bf16-plane split, and for group A
// the LDS-DMA issue of the next k-tile) and a COMPUTE phase (its TM·TN·(PL==3 ? 6 : 1)·2 MFMAs),
// each ended by a workgroup barrier. Group B starts one phase late, so on every SIMD one wave's
// MFMA chain runs while the other wave does its loads and split VALU: the matrix pipe no longer
// waits for the operand work (the glds kernel measured that work and the MFMAs as additive).
// Phase p: A does MEM(p/2) on even p and COMP on odd p; B does MEM on odd and COMP on even p > 0.
// Stages: 2 LDS buffers; group A issues k-tile t+1 during MEM(t) into the buffer k-tile t-1 used
// (group B finished reading it in phase 2t-1), and waits for it (vmcnt 0) at the end of COMP(t),
// before the barrier that opens phase 2t+2 where A first reads it.
template <int TM, int TN, int PL>
__global__ __launch_bounds__(512) void conv_pp_kernel(const ConvArgs p) {
  constexpr int WM = 4, WN = 2;
  constexpr int NT = 512, NL = 256;  // threads, loader threads (group A)
  constexpr int BM = 32 * TM * WM;
  constexpr int BN = 32 * TN * WN;
  constexpr int CA = BM * 8;  // 16-byte chunks of the fp32 A tile (32 k per row)
  constexpr int CB = BN * 4;  // 16-byte chunks of one bf16 B plane
  constexpr int GA = CA / NL;
  constexpr int GB = CB / NL;
  static_assert(GA * NL == CA && GB * NL == CB && GB >= 1, "DMA pieces must tile the loader group");
  constexpr int STAGE = CA + PL * CB;
  constexpr int NS = 2;
  constexpr int NB = (WM * WN * TM * 32 * TN * 32 / 4 <= NS * STAGE) ? TM : 1;
  constexpr int EPI = WM * WN * NB * 32 * TN * 32 / 4;
  constexpr int SMEM = NS * STAGE > EPI ? NS * STAGE : EPI;
  static_assert(SMEM * 16 <= 163840, "LDS");
  __shared__ uint4 smem[SMEM];

  const sp_conv_desc& d = p.d;
  const int64_t wps = d.wt_plane_stride;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const bool grpA = wave < 4;

  const int tilesN = (d.Cout + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int mt = wg / tilesN;
  const int n0 = (wg - mt * tilesN) * BN;
  const int64_t m0 = (int64_t)mt * BM;

  // loader state (group A threads only use it)
  const int lt = tid & (NL - 1);
  const int ca = (lt & 7) ^ (((lt >> 3) >> 1) & 7);
  int a_iy0[GA], a_ix0[GA];
  const float* a_ptr[GA];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int64_t m = m0 + ((j * NL + lt) >> 3);
    const bool ok = m < p.M;
    const int64_t mm = ok ? m : 0;
    const int b = (int)(mm / p.HoWo);
    const int rem = (int)(mm - (int64_t)b * p.HoWo);
    const int oy = rem / d.Wo;
    const int ox = rem - oy * d.Wo;
    a_iy0[j] = ok ? oy * d.stride - d.pad : -(1 << 20);
    a_ix0[j] = ox * d.stride - d.pad;
    a_ptr[j] = d.A + (((int64_t)b * d.H + a_iy0[j]) * d.W + a_ix0[j]) * d.lda + ca * 4;
  }
  const int cbk = (lt & 3) ^ (((lt >> 2) >> 2) & 3);
  const uint16_t* b_ptr[GB];
  bool b_ok[GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int n = n0 + ((j * NL + lt) >> 2);
    b_ok[j] = n < d.Cout;
    b_ptr[j] = d.Wt_bf16 + (int64_t)(b_ok[j] ? n : 0) * p.K + cbk * 8;
  }
  const char* zero = reinterpret_cast<const char*>(g_zero_chunk);

  int s_kh = 0, s_kw = 0, s_c0 = 0;
  const int nk_all = p.K / KT;
  const int kt0 = (int)(((int64_t)nk_all * blockIdx.z) / p.splits);
  const int kt1 = (int)(((int64_t)nk_all * (blockIdx.z + 1)) / p.splits);
  const int nk = kt1 - kt0;
  {
    const int k0 = kt0 * KT;
    const int tap = k0 / d.Cin;
    s_c0 = k0 - tap * d.Cin;
    s_kh = tap / d.KW;
    s_kw = tap - s_kh * d.KW;
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)smem;
  const uint32_t wave_off = (uint32_t)__builtin_amdgcn_readfirstlane((wave & 3) * 64 * 16);
  auto issue = [&](int kt, int buf) {  // group A only
    const uint32_t st = lds0 + (uint32_t)(buf * STAGE * 16) + wave_off;
    const int64_t off = ((int64_t)s_kh * d.W + s_kw) * d.lda + s_c0;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const bool ok = (unsigned)(a_iy0[j] + s_kh) < (unsigned)d.H && (unsigned)(a_ix0[j] + s_kw) < (unsigned)d.W;
      const void* src = ok ? static_cast<const void*>(a_ptr[j] + off) : static_cast<const void*>(zero + ca * 16);
      glds16(src, st + j * NL * 16);
    }
    const int k0 = kt * KT;
#pragma unroll
    for (int pl = 0; pl < PL; ++pl)
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const void* src = b_ok[j] ? static_cast<const void*>(b_ptr[j] + pl * wps + k0)
                                  : static_cast<const void*>(zero + cbk * 16);
        glds16(src, st + (CA + pl * CB + j * NL) * 16);
      }
    s_c0 += KT;
    if (s_c0 >= d.Cin) {
      s_c0 = 0;
      if (++s_kw == d.KW) {
        s_kw = 0;
        ++s_kh;
      }
    }
  };

  const int wm = wave / WN;
  const int wn = wave - wm * WN;
  const int r = lane & 31;
  const int h = lane >> 5;
  int a_row[TM], a_sz[TM], b_row[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    a_row[i] = (wm * TM * 32 + i * 32 + r) * 8;
    a_sz[i] = ((wm * TM * 32 + i * 32 + r) >> 1) & 7;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) b_row[j] = wn * TN * 32 + j * 32 + r;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  bf16x8 fa[2][TM][PL], fb[2][TN][PL];
  auto mem = [&](int buf) {  // fragments of both k16 steps of stage buffer `buf`
    const uint4* st = smem + buf * STAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int pl = 0; pl < PL; ++pl)
          fb[s][j][pl] = *reinterpret_cast<const bf16x8*>(st + CA + pl * CB + sw16(b_row[j], 2 * s + h));
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int c0 = 4 * s + 2 * h;
        const float4 x0 = *reinterpret_cast<const float4*>(st + a_row[i] + (c0 ^ a_sz[i]));
        const float4 x1 = *reinterpret_cast<const float4*>(st + a_row[i] + ((c0 + 1) ^ a_sz[i]));
        split_frag_pk<PL>(x0, x1, fa[s][i]);
      }
    }
  };
  auto comp = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_planes<PL>(fa[s][i], fb[s][j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    raw_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: k-tile 0 landed and visible before anyone's first MEM phase
  if (grpA && nk > 0) {
    issue(kt0, 0);
    wait_vmcnt<0>();
  }
  barrier();
  if (!grpA) barrier();  // group B runs one phase behind
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    // MEM(t)
    if (grpA && t + 1 < nk) issue(kt0 + t + 1, buf ^ 1);
    mem(buf);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this phase's LDS reads are done before the buffer is refilled
    barrier();
    // COMP(t)
    comp();
    if (grpA) wait_vmcnt<0>();  // k-tile t+1 landed before the barrier that opens A's MEM(t+1)
    barrier();
  }
  if (grpA) barrier();  // match group B's extra barrier

  __syncthreads();
  float* smemf = reinterpret_cast<float*>(smem);
  epilogue_tile<TM, TN, NB, false, PL == 1, CNT>(p, smemf + wave * (NB * 32 * TN * 32), acc, m0 + wm * TM * 32,
                                                  n0 + wn * TN * 32, lane);
  if constexpr (CNT) {
    if (p.counters)  // split-K, combined in this launch by the tile's last workgroup
      splitk_combine<NT, BM, BN>(p, reinterpret_cast<int*>(smem), wg, m0, n0);
  }
}

template <int TM, int TN>
int launch_pp(const ConvArgs& a, int planes, hipStream_t s) {
  constexpr int BM = 32 * TM * 4, BN = 32 * TN * 2;
  const int64_t tiles = ((a.M + BM - 1) / BM) * ((a.d.Cout + BN - 1) / BN);
  if (tiles > 0x7fffffff) {
    set_error("sp_conv2d: %lld tiles exceed the grid", (long long)tiles);
    return -1;
  }
  dim3 grid((unsigned)tiles, 1, a.splits);
  if (planes == 3)
    hipLaunchKernelGGL((conv_pp_kernel<TM, TN, 3>), grid, dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL((conv_pp_kernel<TM, TN, 1>), grid, dim3(512), 0, s, a);
  int rc = check_launch(planes == 3 ? "sp_conv2d(f32x3 ping-pong)" : "sp_conv2d(bf16 ping-pong)");
  if (rc || a.splits == 1) return rc;
  return launch_splitk_reduce(a, s);
}


#endif  // SP_DIAG_KERNELS
// The staggered (conv_x3s, cfg 70-72) and persistent (conv_x3p, cfg 73-75) split kernels below hold no tile-table
// entry and lost on every large C2 shape when re-timed in round 5 (1.1-2× the table's tiles,
// profiles/r5/x3/retune_x3s_x3p.json): diagnostic builds only, like conv_pipe / conv_pp above.
#if SP_DIAG_KERNELS
// ---------------------------------------------------------------------------------------------
// Staggered split-GEMM kernel (x3 / bf16): 8 waves, each owning 32 rows × the whole BN = 32·TN
// columns of a 256 × BN tile, so every A fragment is split once per workgroup (VALU per MFMA
// = 44 / (6·TN) instead of 44 / (6·TN) × the waves that share a row band). k advances 16 per LDS
// stage, NS = 4 stages (fp32 A 16 KB + 3 bf16 B planes 24 KB each). Between two barriers a wave
// does two independent things: the MFMAs of step t (A planes split in the previous interval,
// B fragments read now) and the read + split of A for step t+1. Waves 0-3 split first, waves 4-7
// compute first, so on every SIMD one wave's VALU / LDS work runs beside the other's MFMA chain
// instead of both waves doing the same kind of work at the same time. DMA for step t+3 is issued
// right after barrier t into the buffer step t-1 used; it has two intervals to land.
template <int TN, int PL>
__global__ __launch_bounds__(512) void conv_x3s_kernel(const ConvArgs p) {
  constexpr int NT = 512, BM = 256, BN = 32 * TN, BK = 16, NS = 4;
  constexpr int CA = BM * 4;   // 16-byte chunks of the fp32 A stage (4 per row)
  constexpr int CB = 256 * 2;  // chunks of one bf16 B plane (2 per row; 256 rows, rows >= BN zero)
  constexpr int GA = CA / NT;  // 2
  constexpr int GLDS = GA + PL;
  constexpr int STAGE = CA + PL * CB;
  constexpr int EB = TN % 2 == 0 ? TN / 2 : TN;  // epilogue column blocks per round
  constexpr int EPI = 8 * 32 * EB * 32 / 4;
  constexpr int SMEM = NS * STAGE > EPI ? NS * STAGE : EPI;
  static_assert(SMEM * 16 <= 163840, "LDS");
  __shared__ uint4 smem[SMEM];

  const sp_conv_desc& d = p.d;
  const int64_t wps = d.wt_plane_stride;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;

  const int tilesN = (d.Cout + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int mt = wg / tilesN;
  const int n0 = (wg - mt * tilesN) * BN;
  const int64_t m0 = (int64_t)mt * BM;

  // A pieces: tile row (j·NT + tid) / 4, LDS position tid % 4, global chunk (tid % 4) ^ ((row >> 2) & 3)
  const int ca = (tid & 3) ^ ((tid >> 4) & 3);
  int a_iy0[GA], a_ix0[GA];
  const float* a_ptr[GA];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int64_t m = m0 + ((j * NT + tid) >> 2);
    const bool ok = m < p.M;
    const int64_t mm = ok ? m : 0;
    const int b = (int)(mm / p.HoWo);
    const int rem = (int)(mm - (int64_t)b * p.HoWo);
    const int oy = rem / d.Wo;
    const int ox = rem - oy * d.Wo;
    a_iy0[j] = ok ? oy * d.stride - d.pad : -(1 << 20);
    a_ix0[j] = ox * d.stride - d.pad;
    a_ptr[j] = d.A + (((int64_t)b * d.H + a_iy0[j]) * d.W + a_ix0[j]) * d.lda + ca * 4;
  }
  // B piece (one per plane): tile row tid / 2, global chunk (tid & 1) ^ ((row >> 3) & 1)
  const int cbk = (tid & 1) ^ ((tid >> 4) & 1);
  const int brow_ld = tid >> 1;
  const bool b_ok = brow_ld < BN && n0 + brow_ld < d.Cout;
  const uint16_t* b_ptr = d.Wt_bf16 + (int64_t)(b_ok ? n0 + brow_ld : 0) * p.K + cbk * 8;
  const char* zero = reinterpret_cast<const char*>(g_zero_chunk);

  int s_kh = 0, s_kw = 0, s_c0 = 0;
  const int nk_all = p.K / BK;
  const int kt0 = (int)(((int64_t)nk_all * blockIdx.z) / p.splits);
  const int kt1 = (int)(((int64_t)nk_all * (blockIdx.z + 1)) / p.splits);
  const int nk = kt1 - kt0;
  {
    const int k0 = kt0 * BK;
    const int tap = k0 / d.Cin;
    s_c0 = k0 - tap * d.Cin;
    s_kh = tap / d.KW;
    s_kw = tap - s_kh * d.KW;
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)smem;
  const uint32_t wave_off = (uint32_t)__builtin_amdgcn_readfirstlane(wave * 64 * 16);
  // DMA of one k-step in two halves: issue_prep computes the GLDS source addresses (and advances the
  // tap walk), issue_piece(i) issues piece i — the pieces go out one per MFMA block inside mma(), so
  // their issue cost lands in MFMA gaps instead of a DMA burst after the barrier.
  const void* isrc[GLDS];
  uint32_t ist = 0;
  auto issue_prep = [&](int kt, int buf) {
    ist = lds0 + (uint32_t)(buf * STAGE * 16) + wave_off;
    const int64_t off = ((int64_t)s_kh * d.W + s_kw) * d.lda + s_c0;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const bool ok = (unsigned)(a_iy0[j] + s_kh) < (unsigned)d.H && (unsigned)(a_ix0[j] + s_kw) < (unsigned)d.W;
      isrc[j] = ok ? static_cast<const void*>(a_ptr[j] + off) : static_cast<const void*>(zero + ca * 16);
    }
    const int k0 = kt * BK;
#pragma unroll
    for (int pl = 0; pl < PL; ++pl)
      isrc[GA + pl] = b_ok ? static_cast<const void*>(b_ptr + pl * wps + k0) : static_cast<const void*>(zero + cbk * 16);
    s_c0 += BK;
    if (s_c0 >= d.Cin) {
      s_c0 = 0;
      if (++s_kw == d.KW) {
        s_kw = 0;
        ++s_kh;
      }
    }
  };
  auto issue_piece = [&](int i) {
    glds16(isrc[i], ist + (i < GA ? i * NT * 16 : (CA + (i - GA) * CB) * 16));
  };
  auto issue = [&](int kt, int buf) {
    issue_prep(kt, buf);
#pragma unroll
    for (int i = 0; i < GLDS; ++i) issue_piece(i);
  };

  const int r = lane & 31;
  const int h = lane >> 5;
  const int arow = wave * 32 + r;
  const int apos0 = arow * 4 + ((2 * h) ^ ((arow >> 2) & 3));
  const int apos1 = arow * 4 + ((2 * h + 1) ^ ((arow >> 2) & 3));

  f32x16 acc[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[j][q] = 0.f;

  bf16x8 fa[PL];  // A planes of the step whose MFMAs run next
  bf16x8 fn[PL];  // A planes being prepared for the step after
  auto split_a = [&](int buf, bf16x8* out) {
    const uint4* st = smem + buf * STAGE;
    const float4 x0 = *reinterpret_cast<const float4*>(st + apos0);
    const float4 x1 = *reinterpret_cast<const float4*>(st + apos1);
#if SP_X3S_ABL & 2
    bf16x8 raw = __builtin_bit_cast(bf16x8, make_uint4(__float_as_uint(x0.x), __float_as_uint(x0.y),
                                                       __float_as_uint(x1.x), __float_as_uint(x1.y)));
    for (int q = 0; q < PL; ++q) out[q] = raw;
#else
    split_frag_pk<PL>(x0, x1, out);
#endif
  };
  // B fragments double-buffered in registers: block j+1's ds_reads are issued before block j's
  // MFMAs, so each wait covers loads issued one 6-MFMA group (192 cycles) earlier.
  const int bpos0 = r * 2 + (h ^ ((r >> 3) & 1));  // (brow >> 3) & 1 is the same for brow = j·32 + r
  // per block j: the ds_reads of block j+1, then j's MFMAs, then (when this interval issues DMA) DMA
  // piece j — fenced in that order, so each wait covers loads issued one MFMA group earlier and each
  // DMA piece's issue cost sits between MFMAs
  auto mma = [&](int buf, bool dma) {
    const uint4* st = smem + buf * STAGE + CA + bpos0;
    bf16x8 fb[2][PL];
#pragma unroll
    for (int pl = 0; pl < PL; ++pl) fb[0][pl] = *reinterpret_cast<const bf16x8*>(st + pl * CB);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (j + 1 < TN) {
#pragma unroll
        for (int pl = 0; pl < PL; ++pl)
          fb[(j + 1) & 1][pl] = *reinterpret_cast<const bf16x8*>(st + pl * CB + (j + 1) * 64);
      }
      __builtin_amdgcn_sched_barrier(0);
#if SP_X3S_ABL & 4
      for (int pl = 0; pl < PL; ++pl) asm volatile("" ::"v"(fa[pl]), "v"(fb[j & 1][pl]));
#else
      acc[j] = mfma_planes<PL>(fa, fb[j & 1], acc[j]);
#endif
      __builtin_amdgcn_sched_barrier(0);
      if (j < GLDS && dma) issue_piece(j);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = TN; i < GLDS; ++i)
      if (dma) issue_piece(i);
  };

  // prologue: steps 0..2 in flight, step 0 landed, its A planes split
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(kt0 + t, t);
  if (nk > 0) {
    if (nk >= 3) wait_vmcnt<2 * GLDS>();
    else if (nk == 2) wait_vmcnt<GLDS>();
    else wait_vmcnt<0>();
    raw_barrier();
    split_a(0, fa);
  }
  const bool first_split = wave < 4;
#if SP_X3S_STAMP
  const bool stamp_wg = blockIdx.x == 0 && blockIdx.z == 0 && lane == 0;
#define X3S_STAMP(k)                                                                          \
  do {                                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                        \
    if (stamp_wg && t < 64) g_x3s_stamps[(wave * 64 + t) * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                        \
  } while (0)
#else
#define X3S_STAMP(k) \
  do {               \
  } while (0)
#endif
  for (int t = 0; t < nk; ++t) {
    X3S_STAMP(0);
    // step t+1 landed (steps up to t+2 issued: one step may stay in flight)
    if (t + 2 < nk) wait_vmcnt<GLDS>();
    else wait_vmcnt<0>();
    X3S_STAMP(1);
    __builtin_amdgcn_sched_barrier(0);
#if !(SP_X3S_ABL & 8)
    raw_barrier();  // everyone is past interval t-1: buffer (t-1) % 4 is free
#endif
    __builtin_amdgcn_sched_barrier(0);
    X3S_STAMP(2);
#if !(SP_X3S_ABL & 1)
    const bool dma = t + NS - 1 < nk;
    if (dma) issue_prep(kt0 + t + NS - 1, (t + NS - 1) % NS);
#else
    const bool dma = false;
#endif
    X3S_STAMP(3);
    const bool more = t + 1 < nk;
    if (first_split) {
      if (more) split_a((t + 1) % NS, fn);
      X3S_STAMP(4);
      __builtin_amdgcn_sched_barrier(0);
      mma(t % NS, dma);
      X3S_STAMP(5);
    } else {
      mma(t % NS, dma);
      X3S_STAMP(4);
      __builtin_amdgcn_sched_barrier(0);
      if (more) split_a((t + 1) % NS, fn);
      X3S_STAMP(5);
    }
#pragma unroll
    for (int pl = 0; pl < PL; ++pl) fa[pl] = fn[pl];
  }

  __syncthreads();  // every wave done reading the stages before the epilogue reuses the LDS
  float* region = reinterpret_cast<float*>(smem) + wave * (32 * EB * 32);
  constexpr int W = EB * 32;
  const sp_conv_desc& dd = p.d;
  const bool fastv = p.vec_epi && p.splits == 1;
  const int64_t mb = m0 + wave * 32;
#pragma unroll
  for (int j0 = 0; j0 < TN; j0 += EB) {
    if (j0) __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < EB; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) region[((q & 3) + 8 * (q >> 2) + 4 * h) * W + j * 32 + r] = acc[j0 + j][q];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    constexpr int PER = 32 * (W / 4) / 64;
    constexpr int G = PER < 4 ? PER : 4;
    static_assert(PER % G == 0, "task groups");
    for (int t0 = 0; t0 < PER; t0 += G) {
      float4 r1[G];
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int cidx = lane + 64 * (t0 + u);
        const int row = cidx / (W / 4);
        const int col = (cidx - row * (W / 4)) * 4;
        const int64_t m = mb + row;
        const int n = n0 + j0 * 32 + col;
        r1[u] = (fastv && dd.res1 && m < p.M && n < dd.Cout) ? *reinterpret_cast<const float4*>(dd.res1 + m * dd.ldr1 + n)
                                                              : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int cidx = lane + 64 * (t0 + u);
        const int row = cidx / (W / 4);
        const int col = (cidx - row * (W / 4)) * 4;
        const int64_t m = mb + row;
        const int n = n0 + j0 * 32 + col;
        if (m >= p.M || n >= dd.Cout) continue;
        const float4 v = *reinterpret_cast<const float4*>(region + row * W + col);
        if (p.splits > 1) {
          store_partial<false>(p, m, n, v);
        } else if (fastv) {
          epilogue_vec(p, m, n, v, r1[u]);
        } else {
          epilogue_store(p, m, n, v);
        }
      }
    }
  }
}

template <int TN>
int launch_x3s(const ConvArgs& a, int planes, hipStream_t s) {
  if (a.d.Cin % 16 || a.K % 16) {
    set_error("sp_conv2d: staggered kernel needs Cin %% 16 == 0 (Cin=%d)", a.d.Cin);
    return -1;
  }
  constexpr int BN = 32 * TN;
  const int64_t tiles = ((a.M + 255) / 256) * ((a.d.Cout + BN - 1) / BN);
  if (tiles > 0x7fffffff) {
    set_error("sp_conv2d: %lld tiles exceed the grid", (long long)tiles);
    return -1;
  }
  dim3 grid((unsigned)tiles, 1, a.splits);
  if (planes == 3)
    hipLaunchKernelGGL((conv_x3s_kernel<TN, 3>), grid, dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL((conv_x3s_kernel<TN, 1>), grid, dim3(512), 0, s, a);
  int rc = check_launch(planes == 3 ? "sp_conv2d(f32x3 staggered)" : "sp_conv2d(bf16 staggered)");
  if (rc || a.splits == 1) return rc;
  return launch_splitk_reduce(a, s);
}


// ---------------------------------------------------------------------------------------------
// Persistent staggered split-GEMM kernel (x3 / bf16). The x3s interval structure (8 waves × 32
// rows × BN columns, k16 stages, 4-stage LDS ring, waves 0-3 split-then-MFMA, waves 4-7
// MFMA-then-split), run by one workgroup per CU over a STREAM of (tile, k-step) pairs: the ring
// never drains between tiles, so the next tile's first stages land while the current one
// finishes, and there is no per-tile launch / prologue. The MFMAs compute Cᵀ (weights as the
// first operand, activations as the second), which leaves every lane holding 4-channel groups
// of one output pixel: the fused epilogue goes straight from registers to float4 loads / stores
// (no LDS staging), so its stores drain while the next tile's MFMAs run.
// Tiles are dealt XCD-major: the tiles of XCD x are a contiguous range, taken round-robin by the
// workgroups on that XCD (N fastest), so concurrently running tiles share A row panels in L2.
template <int TN, int PL>
__global__ __launch_bounds__(512) void conv_x3p_kernel(const ConvArgs p, int ntiles) {
  constexpr int NT = 512, BM = 256, BN = 32 * TN, BK = 16, NS = 4;
  constexpr int CA = BM * 4;
  constexpr int CB = 256 * 2;
  constexpr int GA = CA / NT;
  constexpr int GLDS = GA + PL;
  constexpr int STAGE = CA + PL * CB;
  static_assert(NS * STAGE * 16 <= 163840, "LDS");
  __shared__ uint4 smem[NS * STAGE];

  const sp_conv_desc& d = p.d;
  const int64_t wps = d.wt_plane_stride;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int tilesN = (d.Cout + BN - 1) / BN;

  // this workgroup's tiles: XCD-contiguous ranges, round-robin inside the XCD
  const int G = gridDim.x;
  const int xcd = blockIdx.x & 7;
  const int loc = blockIdx.x >> 3;
  const int nloc = (G - xcd + 7) >> 3;  // workgroups with this blockIdx.x % 8
  int before = 0;                        // workgroups in the groups before this one
  for (int y = 0; y < xcd; ++y) before += (G - y + 7) >> 3;
  // group x takes a contiguous tile range in proportion to its workgroups (any grid size)
  const int t_beg = (int)((int64_t)ntiles * before / G);
  const int t_end = (int)((int64_t)ntiles * (before + nloc) / G);
  const int my_tiles = t_end - t_beg > loc ? (t_end - t_beg - loc + nloc - 1) / nloc : 0;
  const int nk = p.K / BK;
  const int total = my_tiles * nk;

  const int ca = (tid & 3) ^ ((tid >> 4) & 3);
  const int cbk = (tid & 1) ^ ((tid >> 4) & 1);
  const int brow_ld = tid >> 1;
  const char* zero = reinterpret_cast<const char*>(g_zero_chunk);

  // issue cursor: the tile / k-step the next DMA belongs to
  int i_tile = 0, i_k = 0, s_kh = 0, s_kw = 0, s_c0 = 0;
  int a_iy0[GA], a_ix0[GA];
  const float* a_ptr[GA];
  bool b_ok = false;
  const uint16_t* b_ptr = nullptr;
  auto set_issue_tile = [&](int ti) {
    const int wg = t_beg + loc + ti * nloc;
    const int mt = wg / tilesN;
    const int n0 = (wg - mt * tilesN) * BN;
    const int64_t m0 = (int64_t)mt * BM;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int64_t m = m0 + ((j * NT + tid) >> 2);
      const bool ok = m < p.M;
      const int64_t mm = ok ? m : 0;
      const int b = (int)(mm / p.HoWo);
      const int rem = (int)(mm - (int64_t)b * p.HoWo);
      const int oy = rem / d.Wo;
      const int ox = rem - oy * d.Wo;
      a_iy0[j] = ok ? oy * d.stride - d.pad : -(1 << 20);
      a_ix0[j] = ox * d.stride - d.pad;
      a_ptr[j] = d.A + (((int64_t)b * d.H + a_iy0[j]) * d.W + a_ix0[j]) * d.lda + ca * 4;
    }
    b_ok = brow_ld < BN && n0 + brow_ld < d.Cout;
    b_ptr = d.Wt_bf16 + (int64_t)(b_ok ? n0 + brow_ld : 0) * p.K + cbk * 8;
    s_kh = s_kw = s_c0 = 0;
  };
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)smem;
  const uint32_t wave_off = (uint32_t)__builtin_amdgcn_readfirstlane(wave * 64 * 16);
  auto issue = [&](int buf) {  // the cursor's k-step into stage `buf`, then advance the cursor
    const uint32_t st = lds0 + (uint32_t)(buf * STAGE * 16) + wave_off;
    const int64_t off = ((int64_t)s_kh * d.W + s_kw) * d.lda + s_c0;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const bool ok = (unsigned)(a_iy0[j] + s_kh) < (unsigned)d.H && (unsigned)(a_ix0[j] + s_kw) < (unsigned)d.W;
      const void* src = ok ? static_cast<const void*>(a_ptr[j] + off) : static_cast<const void*>(zero + ca * 16);
      glds16(src, st + j * NT * 16);
    }
    const int k0 = i_k * BK;
#pragma unroll
    for (int pl = 0; pl < PL; ++pl) {
      const void* src = b_ok ? static_cast<const void*>(b_ptr + pl * wps + k0) : static_cast<const void*>(zero + cbk * 16);
      glds16(src, st + (CA + pl * CB) * 16);
    }
    s_c0 += BK;
    if (s_c0 >= d.Cin) {
      s_c0 = 0;
      if (++s_kw == d.KW) {
        s_kw = 0;
        ++s_kh;
      }
    }
    if (++i_k == nk) {
      i_k = 0;
      if (++i_tile < my_tiles) set_issue_tile(i_tile);
    }
  };

  const int r = lane & 31;
  const int h = lane >> 5;
  const int arow = wave * 32 + r;
  const int apos0 = arow * 4 + ((2 * h) ^ ((arow >> 2) & 3));
  const int apos1 = arow * 4 + ((2 * h + 1) ^ ((arow >> 2) & 3));
  const int bpos0 = r * 2 + (h ^ ((r >> 3) & 1));

  f32x16 acc[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[j][q] = 0.f;

  bf16x8 fa[PL], fn[PL];
  auto split_a = [&](int buf, bf16x8* out) {
    const uint4* st = smem + buf * STAGE;
    const float4 x0 = *reinterpret_cast<const float4*>(st + apos0);
    const float4 x1 = *reinterpret_cast<const float4*>(st + apos1);
    split_frag_pk<PL>(x0, x1, out);
  };
  auto mma = [&](int buf) {  // Cᵀ += W_j · Aᵀ for the 8 (TN) column blocks
    const uint4* st = smem + buf * STAGE + CA + bpos0;
    bf16x8 fb[2][PL];
#pragma unroll
    for (int pl = 0; pl < PL; ++pl) fb[0][pl] = *reinterpret_cast<const bf16x8*>(st + pl * CB);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (j + 1 < TN) {
#pragma unroll
        for (int pl = 0; pl < PL; ++pl)
          fb[(j + 1) & 1][pl] = *reinterpret_cast<const bf16x8*>(st + pl * CB + (j + 1) * 64);
      }
      acc[j] = mfma_planes<PL>(fb[j & 1], fa, acc[j]);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, PL, 0);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (j + 1 < TN) __builtin_amdgcn_sched_group_barrier(0x100, PL, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, PL == 3 ? 6 : 1, 0);
    }
  };
  // fused epilogue straight from the Cᵀ accumulators: lane (r, h) of block j holds pixel m0 + 32·wave + r,
  // channels n0 + 32 j + 8 i + 4 h + {0..3} in acc[j][4i..4i+3]. The activation is a template argument
  // (one straight-line copy per activation) so the unrolled body stays small enough for acc[] to
  // remain in registers.
  auto epi_body = [&](auto act_tag, int64_t m, int n0) {
    constexpr int ACT = decltype(act_tag)::value;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float4 r1[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = n0 + j * 32 + 8 * i + 4 * h;
        r1[i] = (d.res1 && n < d.Cout) ? *reinterpret_cast<const float4*>(d.res1 + m * d.ldr1 + n)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int n = n0 + j * 32 + 8 * i + 4 * h;
        float4 v = make_float4(acc[j][4 * i], acc[j][4 * i + 1], acc[j][4 * i + 2], acc[j][4 * i + 3]);
        if (n < d.Cout) {
          if (d.row_scale) {
            const float rs = d.row_scale[m % d.row_period];
            v.x *= rs; v.y *= rs; v.z *= rs; v.w *= rs;
          }
          const float4 sc = d.scale ? *reinterpret_cast<const float4*>(d.scale + n) : make_float4(1.f, 1.f, 1.f, 1.f);
          const float4 sh = d.shift ? *reinterpret_cast<const float4*>(d.shift + n) : make_float4(0.f, 0.f, 0.f, 0.f);
          v.x = fmaf(v.x, sc.x, sh.x) + r1[i].x; v.y = fmaf(v.y, sc.y, sh.y) + r1[i].y;
          v.z = fmaf(v.z, sc.z, sh.z) + r1[i].z; v.w = fmaf(v.w, sc.w, sh.w) + r1[i].w;
          v.x = act_apply(v.x, ACT); v.y = act_apply(v.y, ACT); v.z = act_apply(v.z, ACT); v.w = act_apply(v.w, ACT);
          if (d.res2) {
            const float4 a2 = *reinterpret_cast<const float4*>(d.res2 + m * d.ldr2 + n);
            v.x += a2.x; v.y += a2.y; v.z += a2.z; v.w += a2.w;
          }
          *reinterpret_cast<float4*>(out_row(d, m) + n) = v;
        }
      }
    }
  };
  auto epilogue = [&](int ti) {
    const int wg = t_beg + loc + ti * nloc;
    const int mt = wg / tilesN;
    const int n0 = (wg - mt * tilesN) * BN;
    const int64_t m = (int64_t)mt * BM + wave * 32 + r;
    if (m < p.M) {
      switch (d.act) {
        case SP_ACT_RELU: epi_body(std::integral_constant<int, SP_ACT_RELU>{}, m, n0); break;
        case SP_ACT_SILU: epi_body(std::integral_constant<int, SP_ACT_SILU>{}, m, n0); break;
        case SP_ACT_GELU: epi_body(std::integral_constant<int, SP_ACT_GELU>{}, m, n0); break;
        default: epi_body(std::integral_constant<int, SP_ACT_NONE>{}, m, n0); break;
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[j][q] = 0.f;
  };

  if (total == 0) return;
  set_issue_tile(0);
  // prologue: stream steps 0..2 in flight, step 0 landed, its A planes split
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < total) issue(t);
  if (total >= 3) wait_vmcnt<2 * GLDS>();
  else if (total == 2) wait_vmcnt<GLDS>();
  else wait_vmcnt<0>();
  raw_barrier();
  split_a(0, fa);
  const bool first_split = wave < 4;
  int c_tile = 0, c_k = 0;  // compute cursor
  for (int t = 0; t < total; ++t) {
    // stream step t+1 landed (steps up to t+2 issued: one may stay in flight). After an epilogue
    // interval that wait already happened before the epilogue's stores were issued (below), so the
    // stores are not waited for here; one interval later they are older than every DMA still
    // allowed in flight and the plain count covers them.
    if (!(c_k == 0 && t > 0)) {
      if (t + 2 < total) wait_vmcnt<GLDS>();
      else wait_vmcnt<0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    raw_barrier();  // everyone is past interval t-1: buffer (t-1) % 4 is free
    __builtin_amdgcn_sched_barrier(0);
    if (t + NS - 1 < total) issue((t + NS - 1) % NS);
    const bool more = t + 1 < total;
    if (first_split) {
      if (more) split_a((t + 1) % NS, fn);
      __builtin_amdgcn_sched_barrier(0);
      mma(t % NS);
    } else {
      mma(t % NS);
      __builtin_amdgcn_sched_barrier(0);
      if (more) split_a((t + 1) % NS, fn);
    }
#pragma unroll
    for (int pl = 0; pl < PL; ++pl) fa[pl] = fn[pl];
    if (++c_k == nk) {
      // the next interval needs step t+2: wait for it now (steps up to t+3 issued), before the
      // epilogue's loads and stores enter the count
      if (t + 3 < total) wait_vmcnt<GLDS>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_sched_barrier(0);
      epilogue(c_tile);
      ++c_tile;
      c_k = 0;
    }
  }
}

template <int TN>
int launch_x3p(const ConvArgs& a, int planes, hipStream_t s) {
  if (a.d.Cin % 16 || a.K % 16 || a.splits != 1 || !a.vec_epi) {
    set_error("sp_conv2d: persistent kernel needs Cin %% 16 == 0, no split-K and 16-byte aligned C / residual "
              "/ BN rows with Cout %% 4 == 0 (Cin=%d Cout=%d)", a.d.Cin, a.d.Cout);
    return -1;
  }
  constexpr int BN = 32 * TN;
  const int64_t tiles = ((a.M + 255) / 256) * ((a.d.Cout + BN - 1) / BN);
  if (tiles > 0x7fffffff) {
    set_error("sp_conv2d: %lld tiles exceed the grid", (long long)tiles);
    return -1;
  }
  const int grid = (int)(tiles < g_num_cus ? tiles : g_num_cus);
  if (planes == 3)
    hipLaunchKernelGGL((conv_x3p_kernel<TN, 3>), dim3(grid), dim3(512), 0, s, a, (int)tiles);
  else
    hipLaunchKernelGGL((conv_x3p_kernel<TN, 1>), dim3(grid), dim3(512), 0, s, a, (int)tiles);
  return check_launch(planes == 3 ? "sp_conv2d(f32x3 persistent)" : "sp_conv2d(bf16 persistent)");
}
#endif  // SP_DIAG_KERNELS (x3s / x3p)

template <int WM, int WN, int TM, int TN>
int launch_cfg(const ConvArgs& a, int planes, hipStream_t s) {
  constexpr int BM = 32 * TM * WM, BN = 32 * TN * WN;
  const int64_t tiles = ((a.M + BM - 1) / BM) * ((a.d.Cout + BN - 1) / BN);
  if (tiles > 0x7fffffff) {
    set_error("sp_conv2d: %lld tiles exceed the grid", (long long)tiles);
    return -1;
  }
  dim3 grid((unsigned)tiles, 1, a.splits);
  ConvArgs b = a;
  b.counters = splitk_counters_for(a, tiles);
  if (b.counters && planes == 3)
    hipLaunchKernelGGL((conv_mfma16_kernel<WM, WN, TM, TN, 3, true, true>), grid, dim3(64 * WM * WN), 0, s, b);
  else if (b.counters)
    hipLaunchKernelGGL((conv_mfma16_kernel<WM, WN, TM, TN, 1, true, true>), grid, dim3(64 * WM * WN), 0, s, b);
  else if (planes == 3)
    hipLaunchKernelGGL((conv_mfma16_kernel<WM, WN, TM, TN, 3, true>), grid, dim3(64 * WM * WN), 0, s, b);
  else
    hipLaunchKernelGGL((conv_mfma16_kernel<WM, WN, TM, TN, 1, true>), grid, dim3(64 * WM * WN), 0, s, b);
  int rc = check_launch(planes == 3 ? "sp_conv2d(f32x3)" : "sp_conv2d(bf16)");
  if (rc || a.splits == 1 || b.counters) return rc;
  return launch_splitk_reduce(a, s);
}

}  // namespace

// cfg (register-staged kernel): 1 = 128×128 (2×2 waves of 64×64), 2 = 256×128 (4×2 waves),
// 3 = 64×128, 4 = 64×64, 5 = 128×256 (2×4 waves), 6 = 128×64;
// cfg (LDS-DMA kernel, no A2): 11 = 128×128 3 stages, 12 = 256×128 2 stages, 13 = 64×128 3 stages,
// 14 = 64×64 3 stages, 15 = 128×256 2 stages, 16 = 128×64 3 stages; < 0 = by shape.
thread_local int g_glds_epv = -1;
void set_glds_epilogue(int v) { g_glds_epv = v; }

int launch_mfma16(const ConvArgs& a, int planes, int cfg, hipStream_t s) {
  if (a.A16) {  // bf16 A planes: the LDS-DMA tiles only (the forced / table tile, else the by-shape rule's)
    // bf16 output rows (the bf16 variant's maps): the slab epilogue ("+ 100" → variant 3: res1 by LDS-DMA,
    // rounded outputs staged as bf16 quads), bit-identical, 1.0-2.1x on every tile measured
    // (profiles/r3/bf16/ab_slab_epilogue_bf16_rows.jsonl; launch_glds falls back where it does not apply)
    const int ep = (planes == 1 && a.d.C_bf16) ? 100 : 0;
    if (cfg >= 11) {
      const int rc = launch_glds_cfg(a, planes, cfg < 100 ? cfg + ep : cfg, s);
      if (rc != -2) return rc;
    }
    int c = -1;
    const auto tiles = [&](int bm, int bn) { return ((a.M + bm - 1) / bm) * ((a.d.Cout + bn - 1) / bn); };
    if (a.d.Cout <= 64) c = tiles(128, 64) >= 192 ? 16 : 14;
    // 3×3s on bf16 rows: 256×128 on 16x16x32 MFMAs beat 256×256 by 1.2-1.3× (profiles/r4/bf16/)
    else if (a.d.KH == 3 && a.d.Cout % 128 == 0 && tiles(256, 128) >= 192) c = 41;
    else if (a.d.Cout % 256 == 0 && a.K >= 512 && tiles(256, 256) >= 192) c = 33;
    else if (a.d.Cout % 128 == 0 && tiles(128, 128) >= 192) c = planes == 3 ? 46 : 45;
    else if (tiles(256, 128) >= 192) c = 12;
    else if (tiles(64, 128) >= 192) c = 13;
    else c = 14;
    const int rc = launch_glds_cfg(a, planes, c + ep, s);
    if (rc == -2) {
      set_error("sp_conv2d: no LDS-DMA tile for bf16 A planes");
      return -1;
    }
    return rc;
  }
  if (!a.fast) {  // generic gather: one small-tile instance per operand mode
    const int64_t tiles = ((a.M + 63) / 64) * ((a.d.Cout + 63) / 64);
    dim3 grid((unsigned)tiles, 1, a.splits);
    if (planes == 3)
      hipLaunchKernelGGL((conv_mfma16_kernel<2, 2, 1, 1, 3, false>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((conv_mfma16_kernel<2, 2, 1, 1, 1, false>), grid, dim3(256), 0, s, a);
    int rc = check_launch(planes == 3 ? "sp_conv2d(f32x3 generic)" : "sp_conv2d(bf16 generic)");
    if (rc || a.splits == 1) return rc;
    return launch_splitk_reduce(a, s);
  }
#if SP_DIAG_KERNELS
  if (cfg >= 70 && cfg <= 75 && (a.d.C_bf16 || a.d.res1_bf16 || a.d.res2_bf16)) cfg = -1;  // register epilogues: fp32 rows only
  if (cfg >= 73 && cfg <= 75 && !a.d.A2 && a.splits == 1 && a.vec_epi) {
    switch (cfg) {
      case 73: return launch_x3p<8>(a, planes, s);  // 256×256 persistent
      case 74: return launch_x3p<6>(a, planes, s);  // 256×192 persistent
      default: return launch_x3p<4>(a, planes, s);  // 256×128 persistent
    }
  }
  if (cfg >= 70 && cfg <= 72 && !a.d.A2) {
    switch (cfg) {
      case 70: return launch_x3s<8>(a, planes, s);  // 256×256
      case 71: return launch_x3s<6>(a, planes, s);  // 256×192
      default: return launch_x3s<4>(a, planes, s);  // 256×128
    }
  }
#else
  if (cfg >= 70 && cfg <= 75 && !a.d.A2) {
    set_error("sp_conv2d: tile configuration %d (conv_x3s / conv_x3p) is in the diagnostic build only", cfg);
    return -1;
  }
#endif
#if SP_DIAG_KERNELS
  if (cfg >= 31 && cfg <= 32 && !a.d.A2) {
    switch (cfg) {
      case 31: return launch_pp<2, 2>(a, planes, s);  // 256×128, waves of 64×64
      default: return launch_pp<1, 2>(a, planes, s);  // 128×128, waves of 32×64
    }
  }
  if (cfg >= 21 && cfg <= 26 && !a.d.A2) {
    switch (cfg) {
      case 21: return launch_pipe<2, 2, 2, 2, 4>(a, planes, s);   // 128×128, 4 stages
      case 22: return launch_pipe<2, 2, 2, 4, 3>(a, planes, s);   // 128×256 (wave 64×128)
      case 23: return launch_pipe<4, 1, 2, 4, 3>(a, planes, s);   // 256×128 (wave 64×128)
      case 24: return launch_pipe<2, 2, 2, 2, 3>(a, planes, s);   // 128×128, 3 stages
      case 25: return launch_pipe<4, 2, 2, 2, 3>(a, planes, s);   // 256×128, 8 waves
      default: return launch_pipe<2, 2, 2, 1, 4>(a, planes, s);   // 128×64, 4 stages
    }
  }
#else
  if (((cfg >= 31 && cfg <= 32) || (cfg >= 21 && cfg <= 26)) && !a.d.A2) {
    set_error("sp_conv2d: tile configuration %d (conv_pipe / conv_pp) is in the diagnostic build only", cfg);
    return -1;
  }
#endif
  // The slab epilogue (conv_glds.h epilogue_tile_rd, "cfg + 100") on the split mode's launches with a BN affine
  // or a residual, for the tiles where it measured faster, bit-identical either way: 1.02-1.28x on the
  // bottleneck expands (the res1 band fetched by LDS-DMA; profiles/r3/x3/ab_residual_dma_epilogue.jsonl),
  // 1.02-1.19x without a residual (the BN constants hoisted per lane; ab_slab_epilogue_nores.jsonl) on tiles
  // 12, 14, 41, 45, 46, 47, 63, 64; 0.59-0.96x on the 256-wide-N / TN = 4 four-wave tiles (33, 44)
  if (planes == 3 && !a.A16 && (a.d.res1 || a.d.scale || a.d.shift) && !a.d.row_scale && a.vec_epi &&
      a.splits == 1 && !a.d.C_bf16 &&
      (cfg == 12 || cfg == 14 || cfg == 41 || cfg == 45 || cfg == 46 || cfg == 47 || cfg == 63 || cfg == 64))
    cfg += g_glds_epv == 4 ? 200 : 100;
  // cfg + 100: the LDS-DMA residual epilogue variant; cfg + 200: its direct-store form
  const int gc = cfg >= 211 && cfg <= 265 ? cfg - 200 : cfg >= 111 && cfg <= 165 ? cfg - 100 : cfg;
  if (((gc >= 11 && gc <= 20) || (gc >= 33 && gc <= 38) || (gc >= 41 && gc <= 51) || (gc >= 62 && gc <= 65)) && !a.d.A2) {
    const int rc = launch_glds_cfg(a, planes, cfg, s);
    if (rc != -2) return rc;
  }
  if (cfg < 0 || (cfg > 6 && cfg < 11) || (cfg > 26 && cfg < 31) || (cfg > 38 && cfg < 41) || (cfg > 51 && cfg < 62) || (cfg > 65 && cfg < 70) || (cfg > 75 && gc == cfg) || (cfg >= 73 && cfg <= 75 && (a.splits > 1 || !a.vec_epi)) || (cfg >= 11 && a.d.A2)) {
    // By shape (tools/conv_bench.py sweeps): the LDS-DMA kernel whenever the operands allow it,
    // the largest tile that still gives >= 192 workgroups, a 64-wide N tile for Cout <= 64;
    // 256×256 where Cout is a multiple of 256 and K >= 512 (+10-16 % there; a 384-wide N wastes
    // half of its second column of tiles, and at K = 256 the 256×128 tile stays ahead).
    const auto tiles = [&](int bm, int bn) { return ((a.M + bm - 1) / bm) * ((a.d.Cout + bn - 1) / bn); };
    const bool dma = !a.d.A2;
    // f32x3, measured (profiles/r1/conv_sweep_2wg_x3.jsonl): short-K wide-N layers (the K = 128 / 256
    // bottleneck expands, the decoder value projection) and 384 / 128-wide outputs on mid-size grids
    // run best with two workgroups per CU (LDS <= 80 KB), where one workgroup's prologue and residual
    // epilogue overlap the other's MFMAs: 1.32× on the stage-3 expand, 1.10× on the CCFM 3×3 @ 40².
    const bool x3 = planes == 3;
    if (a.splits > 1) cfg = 4;
    else if (dma && x3 && a.K <= 256 && a.d.Cout >= 512 && tiles(128, 128) >= 192) cfg = 46;
    else if (dma && x3 && a.d.Cout % 128 == 0 && a.d.Cout % 256 != 0 && a.M >= 40000 &&
             (a.M < 150000 || a.d.Cout == 128) && tiles(128, 128) >= 192) cfg = 45;
    else if (a.d.Cout <= 64)
      cfg = dma ? (x3 && a.d.Cout == 64 && tiles(256, 64) >= 192 ? 51 : (tiles(128, 64) >= 192 ? 16 : 14)) : 4;
    else if (dma && a.d.Cout % 256 == 0 && a.K >= 512 && tiles(256, 256) >= 192) cfg = 33;
    else if (tiles(256, 128) >= 192) cfg = dma ? (a.M >= 150000 ? 41 : 12) : 2;  // tall M: 16x16x32 +6 %
    else if (tiles(64, 128) >= 192) cfg = dma ? 13 : 3;
    else cfg = dma ? 14 : 4;
    if (cfg >= 11) return launch_mfma16(a, planes, cfg, s);
  }
  switch (cfg) {
    case 1: return launch_cfg<2, 2, 2, 2>(a, planes, s);
    case 2: return launch_cfg<4, 2, 2, 2>(a, planes, s);
    case 3: return launch_cfg<2, 2, 1, 2>(a, planes, s);
    case 5: return launch_cfg<2, 4, 2, 2>(a, planes, s);
    case 6: return launch_cfg<2, 2, 2, 1>(a, planes, s);
    default: return launch_cfg<2, 2, 1, 1>(a, planes, s);
  }
}

}  // namespace sp

#if SP_X3S_STAMP
extern "C" int sp_debug_x3s_stamps(void* dst) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(sp::g_x3s_stamps), sizeof(sp::g_x3s_stamps));
}
#endif
