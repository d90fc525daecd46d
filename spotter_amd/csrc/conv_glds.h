// LDS-DMA implicit-GEMM kernel templates on bf16-operand MFMA (x3 split / bf16): the tile
// configurations 11-65 of launch_mfma16 (conv_mfma16.hip), instantiated by conv_glds_p*.hip.
#pragma once
#include "mfma16_common.h"

#ifndef SP_ABLATE
#define SP_ABLATE 0
#endif
// Diagnostic build only (-DSP_GLDS_STAMP): per workgroup (first 16384), wave 0 lane 0 records
// s_memtime at kernel start, when the first k-stage is ready, after the main loop and after the
// epilogue, plus HW_ID (CU / SIMD placement); read back with sp_debug_glds_stamps
// (tools/microbench/glds_stamps.py). Not in the product build.
#ifndef SP_GLDS_STAMP
#define SP_GLDS_STAMP 0
#endif
#ifndef SP_GLDS_ONE_UNIT
#define SP_GLDS_ONE_UNIT 0
#endif

namespace sp {

#if SP_GLDS_STAMP
__device__ unsigned long long g_glds_stamps[16384 * 6];
#define GLDS_STAMP(k)                                                                                 \
  do {                                                                                              \
    __builtin_amdgcn_sched_barrier(0);                                                              \
    if (threadIdx.x == 0 && blockIdx.x < 16384) g_glds_stamps[blockIdx.x * 6 + (k)] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                              \
  } while (0)
#else
#define GLDS_STAMP(k) \
  do {                \
  } while (0)
#endif

// the bf16 slab epilogue's 16-byte store pass (-DSP_EPI16_C8=0: the 8-byte pass everywhere, diagnostic A/B)
#ifndef SP_EPI16_C8
#define SP_EPI16_C8 1
#endif
// -DSP_EPI16_PAIRS=1: its LDS element pass on 4-byte column pairs (DPP swap): measured mixed, off
#ifndef SP_EPI16_PAIRS
#define SP_EPI16_PAIRS 0
#endif

namespace {

template <int WM, int WN, int TM, int TN, int PL, int NS, int BK, int APL = 0>
struct GldsCfg {
  // (64-deep stages were built and measured at 0.70-0.92x of the same wave tile at k32 for both operand
  // modes, profiles/r3/bf16/ab_bk64_*.jsonl: the larger stages cost workgroups per CU; removed in round 4)
  static_assert(BK == 32 || BK == 16, "k per stage");
  static constexpr int NT = 64 * WM * WN;
  static constexpr int BM = 32 * TM * WM;
  static constexpr int BN = 32 * TN * WN;
  // APL: A in memory — 0: fp32 A, split / rounded per fragment; 1: bf16 rows (ConvArgs::A16, bf16 mode)
  static_assert(APL == 0 || APL == PL, "bf16 A planes match the operand mode");
  static constexpr int RA = APL ? BK / 8 : BK / 4;  // 16-byte chunks per A row of one plane
  static constexpr int RB = BK / 8;  // 16-byte chunks per bf16 B row (4 / 2)
  static constexpr int CAP = BM * RA;  // 16-byte chunks of one A plane
  static constexpr int CA = CAP * (APL ? APL : 1);  // ... of the whole A stage
  static constexpr int CB = BN * RB;  // 16-byte chunks of one bf16 B plane
  static constexpr int GAP = CAP / NT;  // DMA pieces per thread per A plane
  static constexpr int GA = CA / NT;
  static constexpr int GB = CB / NT;
  static_assert(GAP * NT == CAP && GB * NT == CB && GB >= 1 && GAP >= 1, "DMA pieces must tile the workgroup");
  static constexpr int GLDS = GA + PL * GB;  // DMA instructions per thread per stage
  static constexpr int STAGE = CA + PL * CB;
  static constexpr int NB = (WM * WN * TM * 32 * TN * 32 / 4 <= NS * STAGE) ? TM : 1;
  static constexpr int EPI = WM * WN * NB * 32 * TN * 32 / 4;
  static constexpr int SMEM = NS * STAGE > EPI ? NS * STAGE : EPI;
  static_assert(NS >= 2 && NS <= 6, "stages");
};

// The LDS-DMA main loop of one output tile: k-tiles [kt0, kt1) of tile `wg` (N fastest) accumulated
// into acc (acc4 for 16x16x32 MFMAs). The caller zeroes the accumulators and owns the epilogue.
// V (variant): 1 = general implicit GEMM (per-piece 64-bit addresses, tap walk, padding selects);
// 2 = the 1×1 fast path (KH = KW = 1, stride 1, no padding, A / weight byte offsets < 4 GiB): per-lane
// 32-bit offsets against SGPR bases that advance by one scalar add per k-step (glds16s); rows past M /
// columns past Cout re-read the last valid row / column (their outputs are masked in the epilogue)
// instead of a zero block. Both split A pair-wise (split_frag_pk). Bit-identical outputs, measured
// 1.02-1.09× over the previous form (element-wise split, general addressing everywhere) on the C2
// shapes (profiles/r3/ab_glds_v2.jsonl, tools/ab_glds.py).
template <int WM, int WN, int TM, int TN, int PL, int NS, int BK, bool M16, int V = 1, int APL = 0>
__device__ __forceinline__ void glds_main(const ConvArgs& p, uint4* smem, int wg, int bi, int kt0, int kt1,
                                          f32x16 (&acc)[TM][TN], f32x4 (&acc4)[M16 ? 2 * TM : 1][M16 ? 2 * TN : 1]) {
  using C = GldsCfg<WM, WN, TM, TN, PL, NS, BK, APL>;
  static_assert(!M16 || BK == 32, "16x16x32 steps need a 32-deep stage");
  constexpr int NT = C::NT, RA = C::RA, RB = C::RB, CA = C::CA, CB = C::CB, GA = C::GA, GB = C::GB;
  constexpr int CAP = C::CAP, GAP = C::GAP;
  constexpr int ES = APL ? 2 : 4;  // bytes per A element
  constexpr int GLDS = C::GLDS, STAGE = C::STAGE, BM = C::BM, BN = C::BN;

  const sp_conv_desc& d = p.d;
  const int64_t wps = d.wt_plane_stride;
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;

  const int tilesN = (d.Cout + BN - 1) / BN;
  const int mt = wg / tilesN;
  const int n0 = (wg - mt * tilesN) * BN;
  const int64_t m0 = (int64_t)mt * BM;
  // the grid matches the problem: every tile starts inside M × Cout, k-tiles inside K, batch member inside batch
  SP_BCHECK(m0, p.M);
  SP_BCHECK(n0, d.Cout);
  SP_BCHECK(bi, p.batch);
  SP_BCHECK((int64_t)kt1 * BK - 1, p.K);
  SP_BCHECK(kt0, kt1);

  // B pieces: row (j·NT + tid) / RB, global chunk (tid % RB) ^ swzB(row): (row >> 2) & 3 at BK = 32
  // (sw16), (row >> 3) & 1 at BK = 16.
  const int cbk = BK == 32 ? (tid & 3) ^ (((tid >> 2) >> 2) & 3) : (tid & 1) ^ (((tid >> 1) >> 3) & 1);
  // A pieces (per plane): piece j of this thread covers tile row (j·NT + tid) / RA, LDS position
  // tid % RA, global chunk (tid % RA) ^ swzA(row) — the same for every j since NT / RA is a multiple of
  // the swizzle period. fp32 A: swzA = (row >> 1) & 7 at BK = 32, (row >> 2) & 3 at BK = 16: either way
  // the 16-lane groups of a fragment read (16 consecutive rows, one chunk) hit 16 distinct bank slots.
  // bf16 A rows: the B rows' swizzle.
  const int ca = APL ? cbk
               : BK == 32 ? (tid & 7) ^ (((tid >> 3) >> 1) & 7) : (tid & 3) ^ (((tid >> 2) >> 2) & 3);
  const char* A = (APL ? reinterpret_cast<const char*>(p.A16) : reinterpret_cast<const char*>(d.A)) +
                  (int64_t)bi * p.bs_a * ES;
  constexpr int NAP = APL ? APL : 1;  // A planes staged
  const int64_t aps = p.a_plane_stride * 2;  // bytes between bf16 A planes
  const uint16_t* Wt = d.Wt_bf16 + (int64_t)bi * p.bs_w;
  int a_iy0[GAP], a_ix0[GAP];
  const char* a_ptr[GAP];
#pragma unroll
  for (int j = 0; j < GAP; ++j) {
    const int64_t m = m0 + (j * NT + tid) / RA;
    const bool ok = m < p.M;
    const int64_t mm = ok ? m : 0;
    const int b = (int)(mm / p.HoWo);
    const int rem = (int)(mm - (int64_t)b * p.HoWo);
    const int oy = rem / d.Wo;
    const int ox = rem - oy * d.Wo;
    SP_BCHECK(b, d.N);
    a_iy0[j] = ok ? oy * d.stride - d.pad : -(1 << 20);
    a_ix0[j] = ox * d.stride - d.pad;
    a_ptr[j] = A + (((int64_t)b * d.H + a_iy0[j]) * d.W + a_ix0[j]) * d.lda * ES + ca * 16;
  }
  const uint16_t* b_ptr[GB];
  bool b_ok[GB];
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int n = n0 + (j * NT + tid) / RB;
    b_ok[j] = n < d.Cout;
    b_ptr[j] = Wt + (int64_t)(b_ok[j] ? n : 0) * p.K + cbk * 8;
  }
  const char* zero = reinterpret_cast<const char*>(g_zero_chunk);
  // V == 2: byte offsets of this lane's A rows / B rows against the operand bases
  uint32_t a_off[V == 2 ? GAP : 1], b_off[V == 2 ? GB : 1];
  if constexpr (V == 2) {
#pragma unroll
    for (int j = 0; j < GAP; ++j) {
      const int64_t m = m0 + (j * NT + tid) / RA;
      a_off[j] = (uint32_t)((m < p.M ? m : p.M - 1) * d.lda * ES + ca * 16);
      SP_BCHECK((m < p.M ? m : p.M - 1) * d.lda + (ca + 1) * (16 / ES) - 1 + (int64_t)(kt1 - 1) * BK,
                (p.M - 1) * d.lda + d.Cin);
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int n = n0 + (j * NT + tid) / RB;
      b_off[j] = (uint32_t)(((int64_t)(n < d.Cout ? n : d.Cout - 1) * p.K + cbk * 8) * 2);
    }
  }

  int s_kh = 0, s_kw = 0, s_c0 = 0;
  const int nk = kt1 - kt0;
  {
    const int k0 = kt0 * BK;
    const int tap = k0 / d.Cin;
    s_c0 = k0 - tap * d.Cin;
    s_kh = tap / d.KW;
    s_kw = tap - s_kh * d.KW;
  }

  // Issue the DMA pieces of k-tile kt into stage buffer `buf`, then advance the tap walk.
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)smem;
  const uint32_t wave_off = (uint32_t)__builtin_amdgcn_readfirstlane(wave * 64 * 16);
  auto issue = [&](int kt, int buf) {
    const uint32_t st = lds0 + (uint32_t)(buf * STAGE * 16) + wave_off;
    if constexpr (V == 2) {
#pragma unroll
      for (int pl = 0; pl < NAP; ++pl) {
        const char* ab = A + pl * aps + (int64_t)kt * BK * ES;
#pragma unroll
        for (int j = 0; j < GAP; ++j) glds16s(a_off[j], ab, st + (pl * CAP + j * NT) * 16);
      }
#pragma unroll
      for (int pl = 0; pl < PL; ++pl) {
        const uint16_t* bb = Wt + pl * wps + (int64_t)kt * BK;
#pragma unroll
        for (int j = 0; j < GB; ++j) glds16s(b_off[j], bb, st + (CA + pl * CB + j * NT) * 16);
      }
      return;
    }
    const int64_t off = (((int64_t)s_kh * d.W + s_kw) * d.lda + s_c0) * ES;
    // the tap walk stays inside the filter and each A piece's channels inside Cin (≤ lda)
    SP_BCHECK(s_kh, d.KH);
    SP_BCHECK(s_c0 + (ca + 1) * (16 / ES) - 1, d.Cin);
#pragma unroll
    for (int j = 0; j < GAP; ++j) {
      const bool ok = (unsigned)(a_iy0[j] + s_kh) < (unsigned)d.H && (unsigned)(a_ix0[j] + s_kw) < (unsigned)d.W;
#pragma unroll
      for (int pl = 0; pl < NAP; ++pl) {
        const void* src = ok ? static_cast<const void*>(a_ptr[j] + pl * aps + off)
                             : static_cast<const void*>(zero + ca * 16);
        glds16(src, st + (pl * CAP + j * NT) * 16);
      }
    }
    const int k0 = kt * BK;
    SP_BCHECK(k0 + cbk * 8 + 7, p.K);
#pragma unroll
    for (int pl = 0; pl < PL; ++pl)
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const void* src = b_ok[j] ? static_cast<const void*>(b_ptr[j] + pl * wps + k0)
                                  : static_cast<const void*>(zero + cbk * 16);
        glds16(src, st + (CA + pl * CB + j * NT) * 16);
      }
    s_c0 += BK;
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

  // M16: each 32×32 block of the wave as 2×2 blocks of v_mfma_f32_16x16x32_bf16 (lane l: A row l & 15,
  // B column l & 15, k = 8(l >> 4) + j; C rows 4(l >> 4) + reg, column l & 15) on the same LDS images.
  auto compute = [&](int buf) {
    const uint4* st = smem + buf * STAGE;
    if constexpr (M16) {
      const int c16 = lane & 15, g = lane >> 4;
      bf16x8 fb[2 * TN][PL];
#pragma unroll
      for (int j = 0; j < 2 * TN; ++j) {
        const int brow = wn * TN * 32 + j * 16 + c16;
#pragma unroll
        for (int pl = 0; pl < PL; ++pl)
          fb[j][pl] = *reinterpret_cast<const bf16x8*>(st + CA + pl * CB + sw16(brow, g));
      }
#pragma unroll
      for (int i = 0; i < 2 * TM; ++i) {
        const int row = wm * TM * 32 + i * 16 + c16;
        bf16x8 fa[PL];
        if constexpr (APL) {
#pragma unroll
          for (int pl = 0; pl < PL; ++pl) fa[pl] = *reinterpret_cast<const bf16x8*>(st + pl * CAP + sw16(row, g));
        } else {
          const int sz = (row >> 1) & 7;
          const float4 x0 = *reinterpret_cast<const float4*>(st + row * RA + ((2 * g) ^ sz));
          const float4 x1 = *reinterpret_cast<const float4*>(st + row * RA + ((2 * g + 1) ^ sz));
          split_frag_pk<PL>(x0, x1, fa);
        }
#pragma unroll
        for (int j = 0; j < 2 * TN; ++j) acc4[i][j] = mfma16x16_planes<PL>(fa, fb[j], acc4[i][j]);
      }
      return;
    }
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 fb[TN][PL];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int brow = wn * TN * 32 + j * 32 + r;
        const int bpos = BK == 32 ? sw16(brow, 2 * s + h) : brow * 2 + (h ^ ((brow >> 3) & 1));
#pragma unroll
        for (int pl = 0; pl < PL; ++pl)
          fb[j][pl] = *reinterpret_cast<const bf16x8*>(st + CA + pl * CB + bpos);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * TM * 32 + i * 32 + r;
        bf16x8 fa[PL];
        if constexpr (APL) {
          const int apos = BK == 32 ? sw16(row, 2 * s + h) : row * 2 + (h ^ ((row >> 3) & 1));
#pragma unroll
          for (int pl = 0; pl < PL; ++pl) fa[pl] = *reinterpret_cast<const bf16x8*>(st + pl * CAP + apos);
        } else {
        const int sz = BK == 32 ? (row >> 1) & 7 : (row >> 2) & 3;
        const int c0 = 4 * s + 2 * h;
        const float4 x0 = *reinterpret_cast<const float4*>(st + row * RA + (c0 ^ sz));
        const float4 x1 = *reinterpret_cast<const float4*>(st + row * RA + ((c0 + 1) ^ sz));
#if SP_ABLATE == 2  // no split: one cvt, planes aliased (same MFMA count)
        {
          bf16x8 hh;
          hh[0] = (__bf16)x0.x; hh[1] = (__bf16)x0.y; hh[2] = (__bf16)x0.z; hh[3] = (__bf16)x0.w;
          hh[4] = (__bf16)x1.x; hh[5] = (__bf16)x1.y; hh[6] = (__bf16)x1.z; hh[7] = (__bf16)x1.w;
          for (int q = 0; q < PL; ++q) fa[q] = hh;
        }
#else
        split_frag_pk<PL>(x0, x1, fa);
#endif
        }
#if SP_ABLATE == 3  // no MFMA: keep the operands alive
#pragma unroll
        for (int j = 0; j < TN; ++j)
          for (int q = 0; q < PL; ++q) asm volatile("" ::"v"(fa[q]), "v"(fb[j][q]));
#else
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_planes<PL>(fa, fb[j], acc[i][j]);
#endif
      }
    }
  };

  // Prologue: stages 0 .. NS-2 in flight.
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(kt0 + t, t);
  for (int kt = 0; kt < nk; ++kt) {
    // retire stage kt: stages kt+1 .. min(kt+NS-2, nk-1) may stay in flight
    const int ahead = (nk - 1 - kt) < (NS - 2) ? (nk - 1 - kt) : (NS - 2);
    if (NS >= 6 && ahead >= 4) wait_vmcnt<(NS >= 6 ? 4 * GLDS : 0)>();
    else if (NS >= 5 && ahead >= 3) wait_vmcnt<(NS >= 5 ? 3 * GLDS : 0)>();
    else if (NS >= 4 && ahead >= 2) wait_vmcnt<(NS >= 4 ? 2 * GLDS : 0)>();
    else if (NS >= 3 && ahead >= 1) wait_vmcnt<(NS >= 3 ? GLDS : 0)>();
    else wait_vmcnt<0>();
    raw_barrier();
    if (kt == 0) GLDS_STAMP(1);
#if SP_ABLATE == 1  // no DMA in the loop (compute on stale stages)
    if (false)
#else
    if (kt + NS - 1 < nk)
#endif
      issue(kt0 + kt + NS - 1, (kt + NS - 1) % NS);
    compute(kt % NS);
  }
}

template <int TM, int TN, bool M16>
__device__ __forceinline__ void glds_zero(f32x16 (&acc)[TM][TN], f32x4 (&acc4)[M16 ? 2 * TM : 1][M16 ? 2 * TN : 1]) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
  if constexpr (M16) {
#pragma unroll
    for (int i = 0; i < 2 * TM; ++i)
#pragma unroll
      for (int j = 0; j < 2 * TN; ++j) acc4[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

// Residual epilogue with the res1 tile fetched by LDS-DMA (variant 2, `EPV`): the plain epilogue fetches
// res1 as float4 loads four tasks at a time, a latency chain that the short-K residual GEMMs (the
// bottleneck expands) spend most of their epilogue in. Here each wave DMAs its whole residual band (32
// rows × 32·TN columns, row-major, lane-linear 16-byte pieces: no VGPRs) into its own LDS slab, combines
// it with the accumulators in the MFMA layout (BN affine, + res1, act: epilogue_vec's order, so the
// result is bit-identical), writes the sums back into the slab and stores row-major float4s. Without a
// residual the same combine still saves the per-task BN scale / shift loads (one pair per lane and column
// block instead). Used for fp32 res1 (or none) without row_scale; res2 is added in the store pass.
template <int TM, int TN, int NB, bool L16>
__device__ __forceinline__ void epilogue_tile_rd(const ConvArgs& p, float* region, f32x16 (*acc)[TN], int64_t mb,
                                                 int nb, int lane) {
  constexpr int WN = TN * 32;
  constexpr int C4 = WN / 4;               // float4 columns per slab row
  constexpr int NI = NB * 32 * C4 / 64;    // 1 KB DMA pieces (and float4 store tasks) per lane per round
  constexpr int NCOL = L16 ? 2 : 1;        // distinct accumulator columns of a lane per 32-wide block
  const sp_conv_desc& d = p.d;
  const int r = lane & 31, h = lane >> 5;
  float scv[TN][NCOL], shv[TN][NCOL];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int k = 0; k < NCOL; ++k) {
      const int n = nb + j * 32 + (L16 ? 16 * k + (lane & 15) : r);
      const bool ok = n < d.Cout;
      scv[j][k] = ok && d.scale ? d.scale[n] : 1.0f;
      shv[j][k] = ok && d.shift ? d.shift[n] : 0.0f;
    }
  const uint32_t rbase = (uint32_t)__builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)region);
  const char* zero = reinterpret_cast<const char*>(g_zero_chunk);
  const bool res = d.res1 != nullptr;  // without a residual: the same combine, BN constants hoisted per lane
#pragma unroll
  for (int i0 = 0; i0 < TM; i0 += NB) {
    const int64_t mr = mb + i0 * 32;
    if (i0) __builtin_amdgcn_wave_barrier();
#pragma unroll 1
    for (int u = 0; u < (res ? NI : 0); ++u) {  // not unrolled: the accumulators are live, keep addresses out of VGPRs
      const int idx = u * 64 + lane;
      const int row = idx / C4;
      const int n = nb + (idx - row * C4) * 4;
      const int64_t m = mr + row;
      const void* src = (m < p.M && n < d.Cout) ? static_cast<const void*>(d.res1 + m * d.ldr1 + n)
                                                 : static_cast<const void*>(zero);
      glds16(src, rbase + u * 1024);
    }
    if (res) wait_vmcnt<0>();
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int rr = L16 ? 16 * (q >> 3) + 4 * (lane >> 4) + (q & 3) : (q & 3) + 8 * (q >> 2) + 4 * h;
          const int cc = L16 ? 16 * ((q >> 2) & 1) + (lane & 15) : r;
          const int k = L16 ? (q >> 2) & 1 : 0;
          float* slot = region + (i * 32 + rr) * WN + j * 32 + cc;
          float v = fmaf(acc[i0 + i][j][q], scv[j][k], shv[j][k]);
          if (res) v += *slot;
          *slot = act_apply(v, d.act);
          // one element at a time: hoisting the slab reads would hold a second accumulator's worth of VGPRs
          __builtin_amdgcn_sched_barrier(0);
        }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
#pragma unroll 1
    for (int t = 0; t < NI; ++t) {
      const int cidx = lane + 64 * t;
      const int row = cidx / C4;
      const int col = (cidx - row * C4) * 4;
      const int64_t m = mr + row;
      const int n = nb + col;
      if (m >= p.M || n >= d.Cout) continue;
      float4 v = *reinterpret_cast<const float4*>(region + row * WN + col);
      if (d.res2) {
        const float4 a = *reinterpret_cast<const float4*>(d.res2 + m * d.ldr2 + n);
        v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
      }
      store_out4(d, m, n, v);
    }
  }
}

// Variant 4 (round 4): the slab epilogue's residual band by LDS-DMA, but the outputs stored straight from the
// accumulators (the MFMA layout: one dword store per accumulator register, two 128-byte row segments per
// wave-instruction; raw buffer stores, out-of-range rows / columns dropped by the buffer bound) instead of
// back through the slab. The slab is then free as soon as a round's combine has read it, so the next
// round's residual DMA is issued before this round's stores. Its wait stays a full vmcnt(0): the stores share
// the counter with the DMA, and the compiler's own waitcnt model treats mixed loads and stores on one vmcnt as
// unordered, so a count that left the stores in flight would not prove the DMA landed. The results go to a
// local array, not back into the accumulators (writing them in place made hipcc store one register sixteen
// times: every row but the first wrong, tests/test_gpu_kernels.py::test_direct_store_epilogue_bit_identical). Same arithmetic as variant 2: bit-identical. fp32 C
// with plain rows (ldc), res1 fp32 or none, no res2 / row_scale; C span < 2^31 bytes.
template <int TM, int TN, int NB, bool L16>
__device__ __forceinline__ void epilogue_tile_rdd(const ConvArgs& p, float* region, f32x16 (*acc)[TN], int64_t mb,
                                                  int nb, int lane) {
  constexpr int WN = TN * 32;
  constexpr int C4 = WN / 4;
  constexpr int NI = NB * 32 * C4 / 64;
  constexpr int NCOL = L16 ? 2 : 1;
  const sp_conv_desc& d = p.d;
  const int r = lane & 31, h = lane >> 5;
  float scv[TN][NCOL], shv[TN][NCOL];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int k = 0; k < NCOL; ++k) {
      const int n = nb + j * 32 + (L16 ? 16 * k + (lane & 15) : r);
      const bool ok = n < d.Cout;
      scv[j][k] = ok && d.scale ? d.scale[n] : 1.0f;
      shv[j][k] = ok && d.shift ? d.shift[n] : 0.0f;
    }
  const uint32_t rbase = (uint32_t)__builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)region);
  const char* zero = reinterpret_cast<const char*>(g_zero_chunk);
  const bool res = d.res1 != nullptr;
  const int nbytes = (int)(((p.M - 1) * d.ldc + d.Cout) * 4);
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(d.C, 0, nbytes, 0x00020000);
  auto fetch = [&](int64_t mr) {
#pragma unroll 1
    for (int u = 0; u < NI; ++u) {
      const int idx = u * 64 + lane;
      const int row = idx / C4;
      const int n = nb + (idx - row * C4) * 4;
      const int64_t m = mr + row;
      const void* src = (m < p.M && n < d.Cout) ? static_cast<const void*>(d.res1 + m * d.ldr1 + n)
                                                 : static_cast<const void*>(zero);
      glds16(src, rbase + u * 1024);
    }
  };
  if (res) fetch(mb);
#pragma unroll
  for (int i0 = 0; i0 < TM; i0 += NB) {
    float o[NB][TN][16];
    const int64_t mr = mb + i0 * 32;
    if (res) wait_vmcnt<0>();
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int rr = L16 ? 16 * (q >> 3) + 4 * (lane >> 4) + (q & 3) : (q & 3) + 8 * (q >> 2) + 4 * h;
          const int cc = L16 ? 16 * ((q >> 2) & 1) + (lane & 15) : r;
          const int k = L16 ? (q >> 2) & 1 : 0;
          float v = fmaf(acc[i0 + i][j][q], scv[j][k], shv[j][k]);
          if (res) v += region[(i * 32 + rr) * WN + j * 32 + cc];
          o[i][j][q] = act_apply(v, d.act);
        }
    if (res && i0 + NB < TM) {
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the combine's slab reads are done
      __builtin_amdgcn_wave_barrier();
      fetch(mr + NB * 32);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int rr = L16 ? 16 * (q >> 3) + 4 * (lane >> 4) + (q & 3) : (q & 3) + 8 * (q >> 2) + 4 * h;
          const int cc = L16 ? 16 * ((q >> 2) & 1) + (lane & 15) : r;
          const int64_t m = mr + i * 32 + rr;
          const int n = nb + j * 32 + cc;
          const int off = (m < p.M && n < d.Cout) ? (int)((m * d.ldc + n) * 4) : 0x7ffffffc;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, o[i][j][q]), crs, off, 0, 0);
        }
  }
}

// The same slab epilogue for bf16 rows (variant 3: the bf16 variant, C_bf16 out, res1_bf16 or no residual, no
// res2): the wave's slab (4 bytes per accumulator) holds the residual band as bf16 in its first half (LDS-DMA,
// 16-byte pieces of 8 channels) and the rounded outputs in its second half; the store pass writes 16-byte
// pieces of 8 channels where Cout, ldc and the output base allow, else 8-byte quads. Same arithmetic and rounding as epilogue_vec + store_out4: bit-identical.
template <int TM, int TN, int NB, bool L16>
__device__ __forceinline__ void epilogue_tile_rd16(const ConvArgs& p, float* region, f32x16 (*acc)[TN], int64_t mb,
                                                   int nb, int lane) {
  constexpr int WN = TN * 32;
  constexpr int NI = NB * 32 * WN / 8 / 64;  // 16-byte residual pieces per lane per round
  constexpr int NQ = NB * 32 * WN / 4 / 64;  // 8-byte output quads per lane per round
  constexpr int NCOL = L16 ? 2 : 1;
  static_assert(NI * 64 * 8 == NB * 32 * WN && NQ * 64 * 4 == NB * 32 * WN, "slab pieces");
  const sp_conv_desc& d = p.d;
  const int r = lane & 31, h = lane >> 5;
  float scv[TN][NCOL], shv[TN][NCOL];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int k = 0; k < NCOL; ++k) {
      const int n = nb + j * 32 + (L16 ? 16 * k + (lane & 15) : r);
      const bool ok = n < d.Cout;
      scv[j][k] = ok && d.scale ? d.scale[n] : 1.0f;
      shv[j][k] = ok && d.shift ? d.shift[n] : 0.0f;
    }
  uint16_t* res16 = reinterpret_cast<uint16_t*>(region);
  uint16_t* out16 = res16 + NB * 32 * WN;
  const uint32_t rbase = (uint32_t)__builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)region);
  const char* zero = reinterpret_cast<const char*>(g_zero_chunk);
  const bool res = d.res1_bf16 != nullptr;
  const bool c8 = SP_EPI16_C8 && d.Cout % 8 == 0 && d.ldc % 8 == 0 && (reinterpret_cast<uintptr_t>(d.C_bf16) & 15) == 0 &&
                  (d.out_rows_per_group <= 0 || d.out_group_stride % 8 == 0);
#pragma unroll
  for (int i0 = 0; i0 < TM; i0 += NB) {
    const int64_t mr = mb + i0 * 32;
    if (i0) __builtin_amdgcn_wave_barrier();
#pragma unroll 1
    for (int u = 0; u < (res ? NI : 0); ++u) {
      const int idx = u * 64 + lane;
      const int row = idx / (WN / 8);
      const int n = nb + (idx - row * (WN / 8)) * 8;
      const int64_t m = mr + row;
      const void* src = (m < p.M && n < d.Cout) ? static_cast<const void*>(d.res1_bf16 + m * d.ldr1 + n)
                                                 : static_cast<const void*>(zero);
      glds16(src, rbase + u * 1024);
    }
    if (res) wait_vmcnt<0>();
#if SP_EPI16_PAIRS
    // Lanes l and l ^ 1 hold adjacent columns of the same rows, and elements q, q + 1 (q even) adjacent rows:
    // one DPP swap per element pair gives the even lane row rr (columns cc, cc + 1) and the odd lane row rr + 1
    // (columns cc - 1, cc), so the residual is read and the output written as 4-byte pairs.
    const bool odd = lane & 1;
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 16; q += 2) {
          const int rr = L16 ? 16 * (q >> 3) + 4 * (lane >> 4) + (q & 3) : (q & 3) + 8 * (q >> 2) + 4 * h;
          const int cc = L16 ? 16 * ((q >> 2) & 1) + (lane & 15) : r;
          const int k = L16 ? (q >> 2) & 1 : 0;
          const float a0 = fmaf(acc[i0 + i][j][q], scv[j][k], shv[j][k]);
          const float a1 = fmaf(acc[i0 + i][j][q + 1], scv[j][k], shv[j][k]);
          const float got = __builtin_bit_cast(
              float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, odd ? a0 : a1), 0xb1, 0xf, 0xf, false));
          float lo = odd ? got : a0, hi = odd ? a1 : got;
          const int pos = (i * 32 + rr + odd) * WN + j * 32 + cc - odd;
          if (res) {
            const uint32_t rp = *reinterpret_cast<const uint32_t*>(res16 + pos);
            lo += bf16_lo(rp);
            hi += bf16_lo(rp >> 16);
          }
          *reinterpret_cast<uint32_t*>(out16 + pos) = pack_bf16x2(act_apply(lo, d.act), act_apply(hi, d.act));
        }
#else
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int rr = L16 ? 16 * (q >> 3) + 4 * (lane >> 4) + (q & 3) : (q & 3) + 8 * (q >> 2) + 4 * h;
          const int cc = L16 ? 16 * ((q >> 2) & 1) + (lane & 15) : r;
          const int k = L16 ? (q >> 2) & 1 : 0;
          const int pos = (i * 32 + rr) * WN + j * 32 + cc;
          float v = fmaf(acc[i0 + i][j][q], scv[j][k], shv[j][k]);
          if (res) v += bf16_lo(res16[pos]);
          out16[pos] = (uint16_t)(pack_bf16x2(act_apply(v, d.act), 0.f) & 0xffffu);
        }
#endif
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    if (c8) {  // 16-byte pieces (8 channels) where every row piece is aligned and whole
#pragma unroll 1
      for (int t = 0; t < NQ / 2; ++t) {
        const int cidx = lane + 64 * t;
        const int row = cidx / (WN / 8);
        const int col = (cidx - row * (WN / 8)) * 8;
        const int64_t m = mr + row;
        const int n = nb + col;
        if (m >= p.M || n >= d.Cout) continue;
        *reinterpret_cast<uint4*>(d.C_bf16 + out_off(d, m) + n) = *reinterpret_cast<const uint4*>(out16 + row * WN + col);
      }
      continue;
    }
#pragma unroll 1
    for (int t = 0; t < NQ; ++t) {
      const int cidx = lane + 64 * t;
      const int row = cidx / (WN / 4);
      const int col = (cidx - row * (WN / 4)) * 4;
      const int64_t m = mr + row;
      const int n = nb + col;
      if (m >= p.M || n >= d.Cout) continue;
      *reinterpret_cast<uint2*>(d.C_bf16 + out_off(d, m) + n) = *reinterpret_cast<const uint2*>(out16 + row * WN + col);
    }
  }
}

// Fused epilogue of tile `wg` through the LDS (the caller has synchronised the stages away).
// Batched launches: the caller passes the batch member's own output slab in p.d.C and the tile
// index within that member.
template <int WM, int WN, int TM, int TN, int PL, int NS, int BK, bool M16, int APL, int EPV = 1>
__device__ __forceinline__ void glds_epilogue(const ConvArgs& p, uint4* smem, int wg, f32x16 (&acc)[TM][TN],
                                              f32x4 (&acc4)[M16 ? 2 * TM : 1][M16 ? 2 * TN : 1]) {
  using C = GldsCfg<WM, WN, TM, TN, PL, NS, BK, APL>;  // the kernel's own LDS size decides the band count
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wm = wave / WN;
  const int wn = wave - wm * WN;
  const int tilesN = (p.d.Cout + C::BN - 1) / C::BN;
  const int mt = wg / tilesN;
  const int n0 = (wg - mt * tilesN) * C::BN;
  const int64_t m0 = (int64_t)mt * C::BM;
  float* smemf = reinterpret_cast<float*>(smem);
  if constexpr (M16) {
    // 16×16 blocks → the f32x16 of their 32×32 block: element q = 8·bi + 4·bj + reg
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][j][q] = acc4[2 * i + (q >> 3)][2 * j + ((q >> 2) & 1)][q & 3];
  }
  float* region = smemf + wave * (C::NB * 32 * TN * 32);
  // EPV 2 kernels carry only the residual-DMA epilogue (launch_glds checks its conditions on the host): a
  // runtime choice between the two made hipcc read all accumulators out of the AGPRs ahead of the branch
  if constexpr (EPV == 2)
    epilogue_tile_rd<TM, TN, C::NB, M16>(p, region, acc, m0 + wm * TM * 32, n0 + wn * TN * 32, lane);
  else if constexpr (EPV == 3)
    epilogue_tile_rd16<TM, TN, C::NB, M16>(p, region, acc, m0 + wm * TM * 32, n0 + wn * TN * 32, lane);
  else if constexpr (EPV == 4)
    epilogue_tile_rdd<TM, TN, C::NB, M16>(p, region, acc, m0 + wm * TM * 32, n0 + wn * TN * 32, lane);
  else
    epilogue_tile<TM, TN, C::NB, M16, PL == 1>(p, region, acc, m0 + wm * TM * 32, n0 + wn * TN * 32, lane);
}

// OCC: minimum waves per SIMD the register allocation must allow (1 = unconstrained). Applied to the
// 1×1 fast-path instantiations only (launch_glds): the general path's extra address registers spill.
template <int WM, int WN, int TM, int TN, int PL, int NS, int BK, bool M16, int V = 1, int OCC = 1, int APL = 0,
          int EPV = 1>
__global__ __launch_bounds__(64 * WM * WN, OCC) void conv_glds_kernel(const ConvArgs p) {
  using C = GldsCfg<WM, WN, TM, TN, PL, NS, BK, APL>;
  __shared__ uint4 smem[C::SMEM];
  GLDS_STAMP(0);
  int wg = xcd_index(blockIdx.x, gridDim.x);
  // batched launch (Winograd components): member bi owns tiles [bi·tiles_per_batch, (bi+1)·…)
  const int bi = p.batch > 1 ? wg / p.tiles_per_batch : 0;
  wg -= bi * p.tiles_per_batch;
  const int nk_all = p.K / BK;
  const int kt0 = (int)(((int64_t)nk_all * blockIdx.z) / p.splits);
  const int kt1 = (int)(((int64_t)nk_all * (blockIdx.z + 1)) / p.splits);
  f32x16 acc[TM][TN];
  f32x4 acc4[M16 ? 2 * TM : 1][M16 ? 2 * TN : 1];
  glds_zero<TM, TN, M16>(acc, acc4);
  glds_main<WM, WN, TM, TN, PL, NS, BK, M16, V, APL>(p, smem, wg, bi, kt0, kt1, acc, acc4);
  GLDS_STAMP(2);
  __syncthreads();  // every wave done reading the stages before the epilogue reuses the LDS
  ConvArgs q = p;
  q.d.C += (int64_t)bi * p.bs_c;
  glds_epilogue<WM, WN, TM, TN, PL, NS, BK, M16, APL, EPV>(q, smem, wg, acc, acc4);
#if SP_GLDS_STAMP
  __syncthreads();
  GLDS_STAMP(3);
  if (threadIdx.x == 0 && blockIdx.x < 16384) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_glds_stamps[blockIdx.x * 6 + 4] = hw;
    g_glds_stamps[blockIdx.x * 6 + 5] = xcc;
  }
#endif
}

// The 1×1 fast path (V = 2) applies: KH = KW = 1, stride 1, no padding (A row m is A + m·lda), and
// every byte offset of a batch member's A and weight plane fits 32 bits.
inline bool t1_ok(const ConvArgs& a) {
  const sp_conv_desc& d = a.d;
  return d.KH == 1 && d.KW == 1 && d.stride == 1 && d.pad == 0 && d.Ho == d.H && d.Wo == d.W &&
         a.M * d.lda * (a.A16 ? 2 : 4) < (int64_t(1) << 32) && (int64_t)d.Cout * a.K * 2 < (int64_t(1) << 32);
}

// AB: the bf16-A-plane variants (ConvArgs::A16) are compiled for this tile.
template <int WM, int WN, int TM, int TN, int NS, int BK = 32, bool M16 = false, int OCC = 1, bool AB = false>
int launch_glds(const ConvArgs& a, int planes, hipStream_t s, int epv = 1) {
  if (a.d.Cin % BK || a.K % BK) {
    set_error("sp_conv2d: LDS-DMA kernel needs Cin %% %d == 0 (Cin=%d)", BK, a.d.Cin);
    return -1;
  }
  constexpr int BM = 32 * TM * WM, BN = 32 * TN * WN;
  const int64_t per = ((a.M + BM - 1) / BM) * ((a.d.Cout + BN - 1) / BN);
  const int64_t tiles = per * a.batch;
  if (tiles > 0x7fffffff || (a.batch > 1 && a.splits > 1)) {
    set_error("sp_conv2d: %lld tiles exceed the grid (or split-K on a batched GEMM)", (long long)tiles);
    return -1;
  }
  // a tile whose stages do not fit the 160 KB LDS for this operand mode is not instantiated
  using C3 = GldsCfg<WM, WN, TM, TN, 3, NS, BK>;
  using C1 = GldsCfg<WM, WN, TM, TN, 1, NS, BK>;
  constexpr bool fit3 = C3::SMEM * 16 <= 163840, fit1 = C1::SMEM * 16 <= 163840;
  constexpr bool fit1a = [] {  // bf16 A rows: the bf16 operand mode only (not instantiated unless AB)
    if constexpr (AB) return GldsCfg<WM, WN, TM, TN, 1, NS, BK, 1>::SMEM * 16 <= 163840;
    else return false;
  }();
  const bool a16 = a.A16 != nullptr;
  if (a16 && (planes == 3 || !fit1a)) return -2;  // no bf16-A form of this tile: the caller picks another
  if ((planes == 3 && !fit3) || (planes != 3 && !(a16 ? fit1a : fit1))) {
    set_error("sp_conv2d: tile configuration not built for %d operand plane(s)%s (LDS or bf16-A variant)", planes,
              a16 ? " with bf16 A planes" : "");
    return -1;
  }
  ConvArgs ab = a;
  ab.tiles_per_batch = (int32_t)per;
  dim3 grid((unsigned)tiles, 1, a.splits);
  // the 1×1 fast path where it applies, else the general implicit GEMM
  const bool t1 = t1_ok(a);
  const dim3 blk(64 * WM * WN);
  // the slab epilogues: fp32 rows (2: res1 fp32 or none) or bf16 rows (3: C_bf16, res1_bf16 or none, no res2);
  // float4 epilogue, no split-K / row_scale
  if (epv >= 2) {
    const sp_conv_desc& d = a.d;
    const bool base = a.vec_epi && a.splits == 1 && !d.row_scale;
    const bool f32ok = base && !d.C_bf16 && !d.res1_bf16 && !d.res2_bf16;
    const bool bf16ok = base && d.C_bf16 && !d.res1 && !d.res2 && !d.res2_bf16 &&
                        (!d.res1_bf16 || ((reinterpret_cast<uintptr_t>(d.res1_bf16) & 15) == 0 && d.ldr1 % 8 == 0));
    // variant 4 (direct stores) on request (epv 4), where its extra conditions hold; else variant 2
    const bool f32dd = f32ok && !d.res2 && d.out_rows_per_group <= 0 &&
                       ((a.M - 1) * d.ldc + d.Cout) * 4 < (int64_t(1) << 31) - 4;
    epv = (epv == 4 && f32dd) ? 4 : f32ok ? 2 : bf16ok ? 3 : 1;
  }
  if constexpr (fit3) {
    if (planes == 3 && !a16 && t1 && epv == 4)
      hipLaunchKernelGGL((conv_glds_kernel<WM, WN, TM, TN, 3, NS, BK, M16, 2, OCC, 0, 4>), grid, blk, 0, s, ab);
    else if (planes == 3 && !a16 && t1 && epv == 2)
      hipLaunchKernelGGL((conv_glds_kernel<WM, WN, TM, TN, 3, NS, BK, M16, 2, OCC, 0, 2>), grid, blk, 0, s, ab);
    else if (planes == 3 && !a16 && t1)
      hipLaunchKernelGGL((conv_glds_kernel<WM, WN, TM, TN, 3, NS, BK, M16, 2, OCC>), grid, blk, 0, s, ab);
    else if (planes == 3 && !a16)
      hipLaunchKernelGGL((conv_glds_kernel<WM, WN, TM, TN, 3, NS, BK, M16, 1>), grid, blk, 0, s, ab);
  }
  if constexpr (fit1) {
    if (planes != 3 && !a16 && t1)
      hipLaunchKernelGGL((conv_glds_kernel<WM, WN, TM, TN, 1, NS, BK, M16, 2, OCC>), grid, blk, 0, s, ab);
    else if (planes != 3 && !a16)
      hipLaunchKernelGGL((conv_glds_kernel<WM, WN, TM, TN, 1, NS, BK, M16, 1>), grid, blk, 0, s, ab);
  }
  if constexpr (fit1a) {
    if (planes != 3 && a16 && t1 && epv == 3)
      hipLaunchKernelGGL((conv_glds_kernel<WM, WN, TM, TN, 1, NS, BK, M16, 2, OCC, 1, 3>), grid, blk, 0, s, ab);
    else if (planes != 3 && a16 && t1)
      hipLaunchKernelGGL((conv_glds_kernel<WM, WN, TM, TN, 1, NS, BK, M16, 2, OCC, 1>), grid, blk, 0, s, ab);
    else if (planes != 3 && a16 && epv == 3)
      hipLaunchKernelGGL((conv_glds_kernel<WM, WN, TM, TN, 1, NS, BK, M16, 1, 1, 1, 3>), grid, blk, 0, s, ab);
    else if (planes != 3 && a16)
      hipLaunchKernelGGL((conv_glds_kernel<WM, WN, TM, TN, 1, NS, BK, M16, 1, 1, 1>), grid, blk, 0, s, ab);
  }
  int rc = check_launch(planes == 3 ? "sp_conv2d(f32x3 glds)" : "sp_conv2d(bf16 glds)");
  if (rc || a.splits == 1) return rc;
  return launch_splitk_reduce(a, s);
}


// The LDS-DMA tile configurations: (id, WM, WN, TM, TN, NS, BK, M16, OCC, AB). Tile BM × BN = 32·TM·WM ×
// 32·TN·WN, WM × WN waves, NS stages of BK-deep k, M16: v_mfma_f32_16x16x32_bf16 blocks, OCC: the
// register budget of the 1×1 fast path (waves per SIMD), AB: bf16-A-plane variants compiled.
#define SP_GLDS_CONFIGS(X)              \
  X(11, 2, 2, 2, 2, 3, 32, false, 1, false)    \
  X(12, 4, 2, 2, 2, 2, 32, false, 1, true)    \
  X(13, 2, 2, 1, 2, 3, 32, false, 1, true)    \
  X(14, 2, 2, 1, 1, 3, 32, false, 1, true)    \
  X(15, 2, 4, 2, 2, 2, 32, false, 1, false)    \
  X(16, 2, 2, 2, 1, 3, 32, false, 1, true)    /* 128×64, 3 stages */ \
  X(17, 4, 1, 2, 4, 2, 32, false, 1, false)    /* 256×128, 4 waves of 64×128 */ \
  X(18, 2, 2, 2, 4, 2, 32, false, 1, false)    /* 128×256, 4 waves of 64×128 */ \
  X(19, 2, 1, 2, 4, 2, 32, false, 1, false)    /* 128×128, 2 waves of 64×128, 2 stages */ \
  X(20, 2, 1, 2, 4, 3, 32, false, 1, false)    /* 128×128, 2 waves of 64×128 */ \
  X(33, 4, 2, 2, 4, 2, 32, false, 1, true)    /* 256×256, 8 waves of 64×128 */ \
  X(34, 2, 4, 4, 2, 2, 32, false, 1, false)    /* 256×256, 8 waves of 128×64 */ \
  X(35, 4, 1, 2, 4, 4, 16, false, 1, false)    /* 256×128, k16 × 4 stages */ \
  X(36, 4, 1, 2, 4, 5, 16, false, 1, false)    /* 256×128, k16 × 5 stages */ \
  X(37, 4, 2, 2, 4, 3, 16, false, 1, false)    /* 256×256, k16 × 3 */ \
  X(38, 4, 2, 2, 4, 4, 16, false, 1, false)    /* 256×256, k16 × 4 */ \
  X(41, 4, 2, 2, 2, 2, 32, true, 1, true)     /* cfg 12 on 16x16x32 MFMAs */ \
  X(42, 4, 2, 2, 4, 2, 32, true, 1, true)     /* cfg 33 on 16x16x32 MFMAs */ \
  X(43, 2, 2, 2, 2, 3, 32, true, 1, false)     /* cfg 11 on 16x16x32 MFMAs */ \
  X(44, 4, 1, 2, 4, 2, 16, false, 1, true)    /* 256×128, 4 waves of 64×128, k16 × 2 */ \
  X(45, 2, 2, 2, 2, 2, 32, false, 1, true)    /* 128×128, k32 × 2 */ \
  X(46, 2, 2, 2, 2, 2, 16, false, 4, true)    /* 128×128, k16 × 2, four workgroups per CU (see below) */ \
  X(47, 2, 2, 2, 2, 2, 32, true, 1, true)     /* cfg 45 on 16x16x32 MFMAs */ \
  X(48, 2, 2, 2, 4, 2, 16, false, 1, false)    /* 128×256, 4 waves of 64×128, k16 × 2 */ \
  X(49, 4, 1, 2, 4, 2, 32, true, 1, false)     /* cfg 17 on 16x16x32 MFMAs */ \
  X(50, 4, 1, 2, 2, 3, 32, false, 1, false)    /* 256×64, k32 × 3 */ \
  X(51, 4, 1, 2, 2, 2, 32, false, 1, true)    /* 256×64, k32 × 2 */ \
  X(62, 4, 1, 1, 8, 2, 32, false, 1, false)    /* 128×256, 4 waves of 32×256 */ \
  X(63, 8, 1, 1, 4, 2, 32, false, 1, true)    /* 256×128, 8 waves of 32×128 */ \
  X(64, 4, 1, 1, 4, 3, 32, false, 1, true)    /* 128×128, 4 waves of 32×128, 3 stages */ \
  X(65, 8, 1, 1, 4, 2, 32, true, 1, false)     /* cfg 63 on 16x16x32 MFMAs */ \
  /* round 4, bf16-row candidates (deeper DMA pipelines; x3 stages do not fit at 256 rows) */ \
  X(52, 4, 2, 2, 2, 3, 32, false, 1, true)    /* 256×128, k32 × 3 */ \
  X(53, 4, 2, 2, 2, 3, 32, true, 1, true)     /* cfg 52 on 16x16x32 MFMAs */ \
  X(54, 4, 2, 2, 2, 4, 32, true, 1, true)     /* 256×128, k32 × 4, 16x16x32 */ \
  X(55, 4, 2, 2, 4, 3, 32, true, 1, true)     /* 256×256, k32 × 3, 16x16x32 */ \
  X(56, 2, 2, 2, 2, 4, 32, true, 1, true)     /* 128×128, k32 × 4, 16x16x32 */
// (round 5 also built 256×256 bf16-row tiles with 4 and 5 stages of 32 KB at one workgroup per CU, for the
// long-K 3x3s: 1.1-2.3× slower than the table's tiles on all 35 C3 / C2-bf16 shapes above 0.3 ms per step,
// 0.71 against 0.61 ms even at 102400×512×4608, profiles/r5/bf16/retune_*_256x256.json. Removed.)
// (round 5 built 224-row tiles — 224×256 with four waves of 224×64, its 16x16x32 form, 224×128 with two
// waves — so the 51200-row C2 GEMMs would fill the 256 CUs in one wave of 229 tiles: 1.2-2.3× slower than
// the table's tiles on all ten 51200-row shapes, profiles/r5/x3/tune_224.json; one wave per SIMD and the
// A split repeated by every wave cost more than the full wave of CUs gains. Removed.)
// cfg 46's OCC = 4: registers for 4 waves per SIMD (four workgroups per CU): bit-identical, 1.02-1.09x
// over the unconstrained allocation (3 per SIMD) on the short-K shapes it serves
// (profiles/r3/x3/ab_glds_occupancy.jsonl); 122 VGPRs, no spill, on the 1×1 fast path (the general path
// would spill: it keeps the unconstrained allocation).

// The configurations are compiled in kGldsParts translation units (conv_glds_p<k>.hip: id % kGldsParts
// == k) so the build runs them in parallel; launch_glds_cfg (conv_glds.hip) dispatches.
constexpr int kGldsParts = 6;

template <int PART>
int glds_part(const ConvArgs& a, int planes, int cfg, hipStream_t s, int epv) {
  switch (cfg) {
#define SP_GLDS_CASE(id, WM, WN, TM, TN, NS, BK, M16, OCC, AB)                          \
  case id:                                                                            \
    if constexpr ((id) % kGldsParts == PART)                                          \
      return launch_glds<WM, WN, TM, TN, NS, BK, M16, OCC, AB>(a, planes, s, epv);        \
    else                                                                              \
      return -2;
    SP_GLDS_CONFIGS(SP_GLDS_CASE)
#undef SP_GLDS_CASE
    default:
      return -2;
  }
}

}  // namespace
}  // namespace sp
