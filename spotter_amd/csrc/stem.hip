// Backbone stem conv 1 (RN:71-114, first RTDetrResNetConvLayer: 3x3 stride 2, Cin 3 → 32, FrozenBN
// M2:748-758, ReLU) read straight from the processor's NCHW pixel_values (IPP:461-462).
//
// K = 27 leaves an implicit GEMM nothing to tile (the MFMA kernels ran it at 12 TF/s, plus an
// NCHW→NHWC pass over the 157 MB batch), so this is a direct VALU convolution: one lane per output
// pixel, the 27 taps in registers, the Cout×27 weights uniform across the wave (scalar-cache loads),
// fmaf chains in the khwc tap order, BN affine + ReLU; the workgroup's NHWC rows go out through LDS
// as coalesced float4 stores.
// Work per image at 640²: 320²·Cout·27·2 FLOP = 177 MFLOP; compulsory bytes 3·640²·4 in +
// 320²·Cout·4 out (18 MB at Cout 32) — the output write bounds it.
#include "common.h"

namespace sp {
namespace {

constexpr int STEM_BLOCK = 256;

// Each lane computes one pixel's CO outputs; the workgroup's 256 consecutive NHWC rows are one
// contiguous span of y, so the results are staged in LDS (row stride CO+4 floats: 16-byte aligned,
// rows spread over the banks) and written back as consecutive float4s across the lanes.
// OT: float (fp32 rows) or uint16_t (bf16 rows, RNE at the store: the bf16 variant, ABI v10).
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b2));
}

template <int CO, typename OT>
__global__ __launch_bounds__(STEM_BLOCK) void stem_conv_nchw_kernel(
    const float* __restrict__ x, const float* __restrict__ wt, const float* __restrict__ scale,
    const float* __restrict__ shift, OT* __restrict__ y, int n, int h, int w, int ho, int wo,
    int relu) {
  constexpr int LD = CO + 4;
  __shared__ float4 tile4[STEM_BLOCK * LD / 4];
  float* tile = reinterpret_cast<float*>(tile4);
  const int64_t p0 = (int64_t)blockIdx.x * STEM_BLOCK;
  const int64_t total = (int64_t)n * ho * wo;
  const int rows = (int)min<int64_t>(STEM_BLOCK, total - p0);
  const int t = threadIdx.x;
  if (t < rows) {
    const int64_t p = p0 + t;
    const int ox = (int)(p % wo);
    const int64_t q = p / wo;
    const int oy = (int)(q % ho);
    const int b = (int)(q / ho);
    const int64_t hw = (int64_t)h * w;
    SP_BCHECK(b, n);
    const float* xb = x + (int64_t)b * 3 * hw;

    float in[27];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int iy = 2 * oy - 1 + kh;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int ix = 2 * ox - 1 + kw;
        const bool ok = (unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w;
        const int64_t off = ok ? (int64_t)iy * w + ix : 0;
#pragma unroll
        for (int ci = 0; ci < 3; ++ci) {
          const float v = xb[ci * hw + off];
          in[(kh * 3 + kw) * 3 + ci] = ok ? v : 0.f;
        }
      }
    }

#pragma unroll
    for (int c0 = 0; c0 < CO; c0 += 4) {
      float a[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float* wr = wt + (c0 + j) * 27;
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 27; ++k) s = fmaf(in[k], wr[k], s);
        s = fmaf(s, scale[c0 + j], shift[c0 + j]);
        a[j] = relu ? fmaxf(s, 0.f) : s;
      }
      *reinterpret_cast<float4*>(tile + t * LD + c0) = make_float4(a[0], a[1], a[2], a[3]);
    }
  }
  __syncthreads();
  constexpr int C4 = CO / 4;
  const int n4 = rows * C4;
  if constexpr (sizeof(OT) == 4) {
    float4* yo = reinterpret_cast<float4*>(y + p0 * CO);
    for (int i = t; i < n4; i += STEM_BLOCK) {
      const int r = i / C4, c = i - r * C4;
      yo[i] = *reinterpret_cast<const float4*>(tile + r * LD + 4 * c);
    }
  } else {
    uint2* yo = reinterpret_cast<uint2*>(y + p0 * CO);
    for (int i = t; i < n4; i += STEM_BLOCK) {
      const int r = i / C4, c = i - r * C4;
      const float4 v = *reinterpret_cast<const float4*>(tile + r * LD + 4 * c);
      yo[i] = make_uint2(pk_bf16(v.x, v.y), pk_bf16(v.z, v.w));
    }
  }
}

}  // namespace
}  // namespace sp

using namespace sp;

namespace sp {
namespace {
template <typename OT>
int stem_launch(const char* what, const float* x, const float* wt, const float* scale, const float* shift, OT* y,
                int n, int h, int w, int cout, int act, void* stream) {
  SP_ARG_CHECK(x && wt && scale && shift && y && n > 0 && h > 0 && w > 0 && (act == 0 || act == 1) &&
                   (cout == 32 || cout == 64),
               "%s: bad args (cout must be 32 or 64, act none/relu)", what);
  const int ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  const int64_t total = (int64_t)n * ho * wo;
  const unsigned grid = (unsigned)((total + STEM_BLOCK - 1) / STEM_BLOCK);
  if (cout == 32)
    hipLaunchKernelGGL((stem_conv_nchw_kernel<32, OT>), dim3(grid), dim3(STEM_BLOCK), 0, as_stream(stream), x, wt,
                       scale, shift, y, n, h, w, ho, wo, act);
  else
    hipLaunchKernelGGL((stem_conv_nchw_kernel<64, OT>), dim3(grid), dim3(STEM_BLOCK), 0, as_stream(stream), x, wt,
                       scale, shift, y, n, h, w, ho, wo, act);
  return check_launch(what);
}
}  // namespace
}  // namespace sp

extern "C" int sp_stem_conv3x3s2_nchw(const float* x, const float* wt, const float* scale, const float* shift,
                                      float* y, int n, int h, int w, int cout, int act, void* stream) {
  return stem_launch("sp_stem_conv3x3s2_nchw", x, wt, scale, shift, y, n, h, w, cout, act, stream);
}

extern "C" int sp_stem_conv3x3s2_nchw_bf16(const float* x, const float* wt, const float* scale, const float* shift,
                                           uint16_t* y, int n, int h, int w, int cout, int act, void* stream) {
  return stem_launch("sp_stem_conv3x3s2_nchw_bf16", x, wt, scale, shift, y, n, h, w, cout, act, stream);
}

// ---------------------------------------------------------------------------------------------
// Stem convs 2 and 3 of the bf16 variant (RN:78-103: 3×3 stride 1 pad 1, Cin 32 → Cout 32 / 64, FrozenBN,
// ReLU) as a direct LDS-halo convolution on bf16 rows (ABI v10). As an implicit GEMM these ran at
// 179 / 361 TF (C3, 26.2 M output rows): K = 288 gives a 64-wide tile little reuse, a 32-wide Cout
// wastes half of it, and every A row is fetched once per tap. Here a workgroup stages its input halo —
// (4·RPW + 2) rows × (64 + 2) pixels × 32 channels, bf16 — and all 9·Cout·32 weights in LDS once, then
// each wave computes RPW output rows × 64 pixels × Cout on v_mfma_f32_32x32x16_bf16 with the roles
// transposed (A = weights [Cout × k], B = pixels [k × 64]): the accumulator of lane (pixel r, half h)
// then holds four runs of 4 consecutive channels of one pixel, stored as 8-byte bf16 quads after the
// BN affine + act (fp32). LDS chunks are swizzled (chunk ^ ((row >> 2) & 3)) so a 16-lane group's
// 16-byte reads of 16 consecutive pixels / channels cover all 64 banks. The next tile's halo is fetched into
// registers while the current one is computed and the BN affine is read from LDS: 2.8-2.9x (Cout 32) and
// 1.4-1.8x (Cout 64) the implicit GEMM (profiles/r3/bf16/ab_stem_c32_direct_prefetch.jsonl) against 1.9x and
// 1.03-1.16x with a synchronous halo load per tile.
namespace sp {
namespace {

typedef __bf16 bf16x8_s __attribute__((ext_vector_type(8)));
typedef float f32x16_s __attribute__((ext_vector_type(16)));

constexpr int C3_TW = 64;  // output pixels per wave row

template <int CO, int RPW>
__global__ __launch_bounds__(256, 2) void conv3x3_c32_bf16_kernel(const uint16_t* __restrict__ x,
                                                                  const uint16_t* __restrict__ w16,
                                                                  const float* __restrict__ scale,
                                                                  const float* __restrict__ shift,
                                                                  uint16_t* __restrict__ y, int nimg, int h, int w,
                                                                  int tiles_x, int tiles_y, int act) {
  constexpr int TH = 4 * RPW, HR = TH + 2, HC = C3_TW + 2;
  constexpr int HALO = HR * HC * 4;  // 16-byte chunks
  constexpr int WCH = 9 * CO * 4;    // 16-byte chunks of the weights
  constexpr int TMN = CO / 32;       // 32-channel blocks
  constexpr int PFN = (HALO + 255) / 256;  // halo chunks per thread
  __shared__ uint4 lds[HALO + WCH];
  __shared__ float aff[2 * CO];  // the BN affine (per-tile global loads of it would wait behind the prefetch)
  uint4* halo = lds;
  uint4* wl = lds + HALO;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // weights: global [CO][9 taps][32 ci] bf16 (the packed [Cout][K] form) → LDS [tap][n][chunk ^ swz(n)], once
  // per workgroup: the grid is persistent (a few workgroups per CU walk the tiles), since per 256-pixel
  // tile the weights are as many bytes as the input halo
  for (int i = tid; i < WCH; i += 256) {
    const int c = i & 3, tn = i >> 2, n = tn / 9, tap = tn - n * 9;
    wl[(tap * CO + n) * 4 + (c ^ ((n >> 2) & 3))] = *reinterpret_cast<const uint4*>(w16 + (int64_t)i * 8);
  }
  if (tid < CO) {
    aff[tid] = scale[tid];
    aff[CO + tid] = shift[tid];
  }
  const int64_t ntiles = (int64_t)nimg * tiles_x * tiles_y;
  // the next tile's halo (rows oy0-1 .. oy0+TH, pixels ox0-1 .. ox0+64, zero outside the map) is fetched into
  // registers while this one is computed: unconditional loads (out-of-map chunks read x[0] and are zeroed
  // at the stash), so nothing waits for them before the MFMAs
  uint4 pf[PFN];
  unsigned okm = 0;
  auto fetch = [&](int64_t t) {
    const int tx = (int)(t % tiles_x);
    t /= tiles_x;
    const int ty = (int)(t % tiles_y);
    const int b = (int)(t / tiles_y);
  SP_BCHECK(b, nimg);
    SP_BCHECK(b, nimg);
    const int oy0 = ty * TH, ox0 = tx * C3_TW;
#pragma unroll
    for (int k = 0; k < PFN; ++k) {
      const int i = tid + k * 256;
      const int c = i & 3, rc = i >> 2, r = rc / HC, col = rc - r * HC;
      const int iy = oy0 - 1 + r, ix = ox0 - 1 + col;
      const bool ok = i < HALO && (unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w;
      const int64_t off = ok ? (((int64_t)b * h + iy) * w + ix) * 32 + c * 8 : 0;
      pf[k] = *reinterpret_cast<const uint4*>(x + off);
      okm = k == 0 ? (unsigned)ok : (okm | ((unsigned)ok << k));
    }
  };
  if ((int64_t)blockIdx.x < ntiles) fetch(blockIdx.x);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  int64_t t = tile;
  const int tx = (int)(t % tiles_x);
  t /= tiles_x;
  const int ty = (int)(t % tiles_y);
  const int b = (int)(t / tiles_y);
  SP_BCHECK(b, nimg);
  const int oy0 = ty * TH, ox0 = tx * C3_TW;
  __syncthreads();  // the previous tile's halo reads are done
#pragma unroll
  for (int k = 0; k < PFN; ++k) {
    const int i = tid + k * 256;
    if (i < HALO) {
      const int c = i & 3, rc = i >> 2, col = rc % HC;
      halo[rc * 4 + (c ^ ((col >> 2) & 3))] = (okm >> k) & 1u ? pf[k] : make_uint4(0u, 0u, 0u, 0u);
    }
  }
  __syncthreads();
  if (tile + gridDim.x < ntiles) fetch(tile + gridDim.x);

  const int r = lane & 31, hh = lane >> 5;
  for (int rr = 0; rr < RPW; ++rr) {
    const int orow = wave * RPW + rr;  // output row within the tile
    f32x16_s acc[TMN][2];
#pragma unroll
    for (int i = 0; i < TMN; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int tap = kh * 3 + kw;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int ch = 2 * s + hh;  // k chunk: ci 16s + 8hh .. +7
          bf16x8_s fa[TMN], fb[2];
#pragma unroll
          for (int i = 0; i < TMN; ++i) {
            const int n = i * 32 + r;
            fa[i] = *reinterpret_cast<const bf16x8_s*>(wl + (tap * CO + n) * 4 + (ch ^ ((n >> 2) & 3)));
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int col = j * 32 + r + kw;
            fb[j] = *reinterpret_cast<const bf16x8_s*>(halo + ((orow + kh) * HC + col) * 4 + (ch ^ ((col >> 2) & 3)));
          }
#pragma unroll
          for (int i = 0; i < TMN; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
      }
    // epilogue: lane (pixel r of block j, half hh) holds channels i·32 + 8g + 4hh .. +3 in acc[i][j][4g .. 4g+3]
    const int oy = oy0 + orow;
    if (oy < h) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ox = ox0 + j * 32 + r;
        if (ox >= w) continue;
        uint16_t* yrow = y + (((int64_t)b * h + oy) * w + ox) * CO;
#pragma unroll
        for (int i = 0; i < TMN; ++i)
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            // one v_permlane32_swap per value pair gives lane hh channels base .. base + 7 (16-byte stores,
            // as in the Cin-64 kernel below): 1.11x / 1.16x per launch at C3 (profiles/r4/bf16/ab_c32_swap.json)
            float v[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][j][8 * p + e]),
                                                               __float_as_uint(acc[i][j][8 * p + 4 + e]), false, false);
              v[e] = __uint_as_float(sw[0]);
              v[4 + e] = __uint_as_float(sw[1]);
            }
            const int base = i * 32 + 16 * p + 8 * hh;
            unsigned pk[4];
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              const float u0 = fmaf(v[e], aff[base + e], aff[CO + base + e]);
              const float u1 = fmaf(v[e + 1], aff[base + e + 1], aff[CO + base + e + 1]);
              pk[e / 2] = pk_bf16(act ? fmaxf(u0, 0.f) : u0, act ? fmaxf(u1, 0.f) : u1);
            }
            *reinterpret_cast<uint4*>(yrow + base) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
          }
      }
    }
  }
  }  // tiles
}

}  // namespace
}  // namespace sp

extern "C" int sp_conv3x3_c32_bf16(const uint16_t* x, const uint16_t* w16, const float* scale, const float* shift,
                                   uint16_t* y, int n, int h, int w, int cout, int act, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(x && w16 && scale && shift && y && n > 0 && h > 0 && w > 0 && (cout == 32 || cout == 64) &&
                   (act == 0 || act == 1) && ((uintptr_t)x & 15) == 0 && ((uintptr_t)w16 & 15) == 0 &&
                   ((uintptr_t)y & 15) == 0,
               "sp_conv3x3_c32_bf16: bad args (Cin 32, Cout 32 or 64, act none/relu, aligned dense bf16 rows)");
  constexpr int RPW = 1;
  const int tiles_x = (w + C3_TW - 1) / C3_TW, tiles_y = (h + 4 * RPW - 1) / (4 * RPW);
  const int64_t tiles = (int64_t)n * tiles_x * tiles_y;
  // persistent grid: as many workgroups as fit on the chip at once (2 per CU at Cout 64, 3 at Cout 32)
  const int64_t cap = (int64_t)g_num_cus * (cout == 32 ? 3 : 2);
  const unsigned grid = (unsigned)(tiles < cap ? tiles : cap);
  if (cout == 32)
    hipLaunchKernelGGL((conv3x3_c32_bf16_kernel<32, RPW>), dim3(grid), dim3(256), 0, as_stream(stream), x,
                       w16, scale, shift, y, n, h, w, tiles_x, tiles_y, act);
  else
    hipLaunchKernelGGL((conv3x3_c32_bf16_kernel<64, RPW>), dim3(grid), dim3(256), 0, as_stream(stream), x,
                       w16, scale, shift, y, n, h, w, tiles_x, tiles_y, act);
  return check_launch("sp_conv3x3_c32_bf16");
}

// ---------------------------------------------------------------------------------------------
// The same two stem convs in the fp32 modes (ABI v10): direct LDS-halo convolution on fp32 rows with
// v_mfma_f32_32x32x2_f32 (exact fp32 products, fp32 accumulate). As fp32-MFMA implicit GEMMs they ran at
// 93 / 106 TF of 157.3 (C2, profiles/r3/conv_detail_c2_fp32_r3g.json). One persistent workgroup per CU,
// eight waves: the workgroup holds all 9·Cout·32 fp32 weights (36 / 72 KB) and one input halo of
// (8 + 2) rows × (64 + 2) pixels × 32 channels (82.5 KB) in LDS; wave v computes output row v of the
// tile (64 pixels × Cout) with the roles transposed as above (A = weights, B = pixels). The next tile's
// halo is fetched into registers while the current one is computed. Channels: lane (r, half hh) reads a
// float4 (4 consecutive channels of chunk 2q + hh) of its weight row and of its pixel; MFMA e of the four
// takes component e, so MFMA e contracts channels 8q + e and 8q + 4 + e. LDS rows are 8 chunks of 16 B,
// swizzled chunk ^ ((row >> 1) & 7): 16 consecutive rows' reads of one chunk land in 16 distinct slots.
namespace sp {
namespace {

typedef float f32x4_s __attribute__((ext_vector_type(4)));

constexpr int F3_TH = 8, F3_HR = F3_TH + 2, F3_HC = C3_TW + 2;
constexpr int F3_HALO = F3_HR * F3_HC * 8;                  // 16-byte chunks of the halo
constexpr int F3_PF = (F3_HALO + 511) / 512;                // halo chunks per thread

__device__ __forceinline__ int f3_swz(int row, int c) { return c ^ ((row >> 1) & 7); }

template <int CO>
__global__ __launch_bounds__(512, 1) void conv3x3_c32_f32_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ wt,
                                                                 const float* __restrict__ scale,
                                                                 const float* __restrict__ shift,
                                                                 float* __restrict__ y, int nimg, int h, int w,
                                                                 int tiles_x, int tiles_y, int act) {
  constexpr int WCH = 9 * CO * 8;  // 16-byte chunks of the weights
  constexpr int TMN = CO / 32;
  __shared__ uint4 lds[F3_HALO + WCH];
  __shared__ float aff[2 * CO];  // the BN affine: per-tile global loads of it would wait behind the prefetch
  uint4* halo = lds;
  uint4* wl = lds + F3_HALO;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (tid < CO) {
    aff[tid] = scale[tid];
    aff[CO + tid] = shift[tid];
  }
  // weights: global [CO][9 taps][32 ci] fp32 (the packed [Cout][K] form) → LDS [tap][n][chunk ^ swz(n)]
  for (int i = tid; i < WCH; i += 512) {
    const int c = i & 7, tn = i >> 3, n = tn / 9, tap = tn - n * 9;
    wl[(tap * CO + n) * 8 + f3_swz(n, c)] = *reinterpret_cast<const uint4*>(wt + (int64_t)i * 4);
  }
  const int64_t ntiles = (int64_t)nimg * tiles_x * tiles_y;
  uint4 pf[F3_PF];
  unsigned okm = 0;  // bit k: pf[k] is inside the map (out-of-map chunks are loaded from x[0] and zeroed at the stash)
  // fetch tile t's halo (rows oy0-1 .. oy0+8, pixels ox0-1 .. ox0+64; zero outside the map) into registers:
  // unconditional loads, so no wait for them is needed before the MFMAs that follow
  auto fetch = [&](int64_t t) {
    const int tx = (int)(t % tiles_x);
    t /= tiles_x;
    const int ty = (int)(t % tiles_y);
    const int b = (int)(t / tiles_y);
  SP_BCHECK(b, nimg);
    SP_BCHECK(b, nimg);
    const int oy0 = ty * F3_TH, ox0 = tx * C3_TW;
#pragma unroll
    for (int k = 0; k < F3_PF; ++k) {
      const int i = tid + k * 512;
      const int c = i & 7, rc = i >> 3, r = rc / F3_HC, col = rc - r * F3_HC;
      const int iy = oy0 - 1 + r, ix = ox0 - 1 + col;
      const bool ok = i < F3_HALO && (unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w;
      const int64_t off = ok ? (((int64_t)b * h + iy) * w + ix) * 32 + c * 4 : 0;
      pf[k] = *reinterpret_cast<const uint4*>(x + off);
      okm = k == 0 ? (unsigned)ok : (okm | ((unsigned)ok << k));
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int k = 0; k < F3_PF; ++k) {
      const int i = tid + k * 512;
      if (i < F3_HALO) {
        const int c = i & 7, rc = i >> 3, col = rc % F3_HC;
        halo[rc * 8 + f3_swz(col, c)] = (okm >> k) & 1u ? pf[k] : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  };
  if ((int64_t)blockIdx.x < ntiles) fetch(blockIdx.x);
  const int r = lane & 31, hh = lane >> 5;

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    __syncthreads();  // the previous tile's halo reads are done
    stash();
    __syncthreads();
    if (tile + gridDim.x < ntiles) fetch(tile + gridDim.x);  // overlaps the MFMAs below
    int64_t t = tile;
    const int tx = (int)(t % tiles_x);
    t /= tiles_x;
    const int ty = (int)(t % tiles_y);
    const int b = (int)(t / tiles_y);
  SP_BCHECK(b, nimg);
    SP_BCHECK(b, nimg);
    const int oy = ty * F3_TH + wave, ox0 = tx * C3_TW;
    f32x16_s acc[TMN][2];
#pragma unroll
    for (int i = 0; i < TMN; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int tap = kh * 3 + kw;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int ch = 2 * q + hh;  // chunk: ci 8q + 4hh .. +3
          f32x4_s fa[TMN], fb[2];
#pragma unroll
          for (int i = 0; i < TMN; ++i) {
            const int n = i * 32 + r;
            fa[i] = *reinterpret_cast<const f32x4_s*>(wl + (tap * CO + n) * 8 + f3_swz(n, ch));
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int col = j * 32 + r + kw;
            fb[j] = *reinterpret_cast<const f32x4_s*>(halo + ((wave + kh) * F3_HC + col) * 8 + f3_swz(col, ch));
          }
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int i = 0; i < TMN; ++i)
#pragma unroll
              for (int j = 0; j < 2; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][e], fb[j][e], acc[i][j], 0, 0, 0);
        }
      }
    // epilogue: lane (pixel r of block j, half hh) holds channels i·32 + 8g + 4hh .. +3 in acc[i][j][4g .. 4g+3]
    if (oy < h) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ox = ox0 + j * 32 + r;
        if (ox >= w) continue;
        float* yrow = y + (((int64_t)b * h + oy) * w + ox) * CO;
#pragma unroll
        for (int i = 0; i < TMN; ++i)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int n0 = i * 32 + 8 * g + 4 * hh;
            float4 v;
            float* vv = &v.x;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float u = fmaf(acc[i][j][4 * g + e], aff[n0 + e], aff[CO + n0 + e]);
              vv[e] = act ? fmaxf(u, 0.f) : u;
            }
            *reinterpret_cast<float4*>(yrow + n0) = v;
          }
      }
    }
  }  // tiles
}

}  // namespace
}  // namespace sp

extern "C" int sp_conv3x3_c32(const float* x, const float* wt, const float* scale, const float* shift, float* y,
                              int n, int h, int w, int cout, int act, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(x && wt && scale && shift && y && n > 0 && h > 0 && w > 0 && (cout == 32 || cout == 64) &&
                   (act == 0 || act == 1) && ((uintptr_t)x & 15) == 0 && ((uintptr_t)wt & 15) == 0 &&
                   ((uintptr_t)y & 15) == 0,
               "sp_conv3x3_c32: bad args (Cin 32, Cout 32 or 64, act none/relu, aligned dense fp32 rows)");
  const int tiles_x = (w + C3_TW - 1) / C3_TW, tiles_y = (h + F3_TH - 1) / F3_TH;
  const int64_t tiles = (int64_t)n * tiles_x * tiles_y;
  const unsigned grid = (unsigned)(tiles < g_num_cus ? tiles : g_num_cus);  // persistent: one per CU
  if (cout == 32)
    hipLaunchKernelGGL((conv3x3_c32_f32_kernel<32>), dim3(grid), dim3(512), 0, as_stream(stream), x, wt, scale,
                       shift, y, n, h, w, tiles_x, tiles_y, act);
  else
    hipLaunchKernelGGL((conv3x3_c32_f32_kernel<64>), dim3(grid), dim3(512), 0, as_stream(stream), x, wt, scale,
                       shift, y, n, h, w, tiles_x, tiles_y, act);
  return check_launch("sp_conv3x3_c32");
}

// ---------------------------------------------------------------------------------------------
// The stage-0 3×3 (Cin 64 → Cout 64) of the bf16 variant on bf16 rows: the Cin-32 kernel above with 64-channel
// rows (8 chunks of 16 B, swizzled chunk ^ ((row >> 1) & 7)), all 9·64·64 bf16 weights (73.7 KB) and an
// (16 + 2) × (32 + 2) × 64 bf16 halo (78.3 KB) in LDS, eight waves, each two output rows × 32 pixels, rows
// ldx / ldy elements apart (the fused bottleneck tail reads this output as a channel slice). Sums the 576-deep k
// in (tap, 16-channel) order with v_mfma_f32_32x32x16_bf16 blocks, as the implicit GEMM does.
// Tiles are 32 pixels wide so the 160- / 320-pixel stage-0 maps tile exactly (64-wide tiles computed 192 columns
// of every 160). Epilogue: lanes r and r + 32 hold alternating 4-channel runs of one pixel; one
// v_permlane32_swap per value pair gives each lane 8 consecutive channels, so the residual is read and the
// output written as 16-byte row pieces (8 loads / stores per lane instead of 16 of 8 bytes); the residual
// (template RES) is fetched once per tile at the start of the epilogue. At C3's shape (bs256 160², 0.48 TFLOP):
// 0.60 / 0.71 ms without / with the residual against 0.70 / 0.91 for 64-wide tiles with 8-byte epilogue accesses
// (profiles/r4/bf16/ab_c64_tw32.json).
// Diagnostic build only (tools/build_diag.sh with UNIT=stem, -DSP_C64_ABL=bits): timing ablations, results wrong
// with any bit set: 1 no output stores (nor residual use), 4 no halo loads from HBM.
#ifndef SP_C64_ABL
#define SP_C64_ABL 0
#endif
namespace sp {
namespace {

constexpr int B6_TH = 16, B6_TW = 32, B6_HR = B6_TH + 2, B6_HC = B6_TW + 2;
constexpr int B6_HALO = B6_HR * B6_HC * 8;    // 16-byte chunks of the halo
constexpr int B6_WCH = 9 * 64 * 8;            // 16-byte chunks of the weights
constexpr int B6_PF = (B6_HALO + 511) / 512;  // halo chunks per thread

template <bool RES>
__global__ __launch_bounds__(512, 1) void conv3x3_c64_bf16_kernel(const uint16_t* __restrict__ x,
                                                                  const uint16_t* __restrict__ w16,
                                                                  const float* __restrict__ scale,
                                                                  const float* __restrict__ shift,
                                                                  uint16_t* __restrict__ y, int64_t ldx,
                                                                  int64_t ldy, const uint16_t* __restrict__ res,
                                                                  int64_t ldr, int nimg, int h, int w, int tiles_x,
                                                                  int tiles_y, int act) {
  __shared__ uint4 lds[B6_HALO + B6_WCH];
  __shared__ float aff[128];
  uint4* halo = lds;
  uint4* wl = lds + B6_HALO;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // weights: global [64][9 taps][64 ci] bf16 → LDS [tap][n][chunk ^ swz(n)]
  for (int i = tid; i < B6_WCH; i += 512) {
    const int c = i & 7, tn = i >> 3, n = tn / 9, tap = tn - n * 9;
    wl[(tap * 64 + n) * 8 + f3_swz(n, c)] = *reinterpret_cast<const uint4*>(w16 + (int64_t)i * 8);
  }
  if (tid < 64) {
    aff[tid] = scale[tid];
    aff[64 + tid] = shift[tid];
  }
  const int64_t ntiles = (int64_t)nimg * tiles_x * tiles_y;
  uint4 pf[B6_PF];
  unsigned okm = 0;
  auto fetch = [&](int64_t t) {
    const int tx = (int)(t % tiles_x);
    t /= tiles_x;
    const int ty = (int)(t % tiles_y);
    const int b = (int)(t / tiles_y);
  SP_BCHECK(b, nimg);
    SP_BCHECK(b, nimg);
    const int oy0 = ty * B6_TH, ox0 = tx * B6_TW;
#pragma unroll
    for (int k = 0; k < B6_PF; ++k) {
      const int i = tid + k * 512;
      const int c = i & 7, rc = i >> 3, r = rc / B6_HC, col = rc - r * B6_HC;
      const int iy = oy0 - 1 + r, ix = ox0 - 1 + col;
      const bool ok = i < B6_HALO && (unsigned)iy < (unsigned)h && (unsigned)ix < (unsigned)w;
      const int64_t off = ok ? (((int64_t)b * h + iy) * w + ix) * ldx + c * 8 : 0;
#if SP_C64_ABL & 4
      pf[k] = make_uint4((unsigned)off, 0u, 0u, 0u);
#else
      pf[k] = *reinterpret_cast<const uint4*>(x + off);
#endif
      okm = k == 0 ? (unsigned)ok : (okm | ((unsigned)ok << k));
    }
  };
  if ((int64_t)blockIdx.x < ntiles) fetch(blockIdx.x);
  const int r = lane & 31, hh = lane >> 5;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    __syncthreads();  // the previous tile's halo reads are done
#pragma unroll
    for (int k = 0; k < B6_PF; ++k) {
      const int i = tid + k * 512;
      if (i < B6_HALO) {
        const int c = i & 7, rc = i >> 3, col = rc % B6_HC;
        halo[rc * 8 + f3_swz(col, c)] = (okm >> k) & 1u ? pf[k] : make_uint4(0u, 0u, 0u, 0u);
      }
    }
    __syncthreads();
    int64_t t = tile;
    const int tx = (int)(t % tiles_x);
    t /= tiles_x;
    const int ty = (int)(t % tiles_y);
    const int b = (int)(t / tiles_y);
  SP_BCHECK(b, nimg);
    SP_BCHECK(b, nimg);
    const int oy0 = ty * B6_TH + 2 * wave, ox = tx * B6_TW + r;
    int64_t pix[2];
    bool in[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      in[j] = oy0 + j < h && ox < w;
      pix[j] = in[j] ? ((int64_t)b * h + oy0 + j) * w + ox : 0;
      if (in[j]) SP_BCHECK(pix[j], (int64_t)nimg * h * w);
    }
    uint4 rq[2][2][2];  // [row j][channel half i][16-channel group p]: this lane's 8 residual channels
    auto fetch_res = [&]() {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int p = 0; p < 2; ++p)
            rq[j][i][p] = *reinterpret_cast<const uint4*>(res + pix[j] * ldr + i * 32 + 16 * p + 8 * hh);
    };
    if (tile + gridDim.x < ntiles) fetch(tile + gridDim.x);  // overlaps the MFMAs below
    f32x16_s acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int tap = kh * 3 + kw;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int ch = 2 * s + hh;  // k chunk: ci 16s + 8hh .. +7
          bf16x8_s fa[2], fb[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int n = i * 32 + r;
            fa[i] = *reinterpret_cast<const bf16x8_s*>(wl + (tap * 64 + n) * 8 + f3_swz(n, ch));
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int col = r + kw;
            fb[j] = *reinterpret_cast<const bf16x8_s*>(halo + ((2 * wave + j + kh) * B6_HC + col) * 8 +
                                                       f3_swz(col, ch));
          }
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
      }
    if constexpr (RES) fetch_res();  // issued here, not ahead of the MFMAs: 32 more live VGPRs there spill
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#if SP_C64_ABL & 1
      if (!(in[j] && acc[0][j][0] == 1234.5f && acc[1][j][15] == -2.25f)) continue;
#endif
      uint16_t* yrow = y + pix[j] * ldy;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          // accumulator element 4g + e of lane (r, hh) is channel i·32 + 8g + 4hh + e: swap the upper half's
          // g = 2p run with the lower half's g = 2p + 1 run, so lane hh holds channels base .. base + 7
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[i][j][8 * p + e]),
                                                             __float_as_uint(acc[i][j][8 * p + 4 + e]), false, false);
            v[e] = __uint_as_float(sw[0]);
            v[4 + e] = __uint_as_float(sw[1]);
          }
          const int base = i * 32 + 16 * p + 8 * hh;
          float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          if constexpr (RES) {  // pre-activation residual (the basic block's shortcut), bf16 rows
            const uint4 q = rq[j][i][p];
            const unsigned qq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              rv[2 * e] = __uint_as_float(qq[e] << 16);
              rv[2 * e + 1] = __uint_as_float(qq[e] & 0xffff0000u);
            }
          }
          unsigned pk[4];
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            float u0 = fmaf(v[e], aff[base + e], aff[64 + base + e]);
            float u1 = fmaf(v[e + 1], aff[base + e + 1], aff[64 + base + e + 1]);
            if constexpr (RES) {
              u0 += rv[e];
              u1 += rv[e + 1];
            }
            pk[e / 2] = pk_bf16(act ? fmaxf(u0, 0.f) : u0, act ? fmaxf(u1, 0.f) : u1);
          }
          if (in[j]) *reinterpret_cast<uint4*>(yrow + base) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        }
    }
  }  // tiles
}

}  // namespace
}  // namespace sp

extern "C" int sp_conv3x3_c64_bf16(const uint16_t* x, int64_t ldx, const uint16_t* w16, const float* scale,
                                   const float* shift, uint16_t* y, int64_t ldy, const uint16_t* res, int64_t ldr,
                                   int n, int h, int w, int act, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(x && w16 && scale && shift && y && n > 0 && h > 0 && w > 0 && (act == 0 || act == 1) &&
                   ldx >= 64 && ldy >= 64 && ldx % 8 == 0 && ldy % 8 == 0 && ((uintptr_t)x & 15) == 0 &&
                   ((uintptr_t)w16 & 15) == 0 && ((uintptr_t)y & 15) == 0 &&
                   (!res || (ldr >= 64 && ldr % 8 == 0 && ((uintptr_t)res & 15) == 0)),
               "sp_conv3x3_c64_bf16: bad args (act none/relu, 16-byte aligned bf16 rows, ld % 8, ld >= 64)");
  const int tiles_x = (w + B6_TW - 1) / B6_TW, tiles_y = (h + B6_TH - 1) / B6_TH;
  const int64_t tiles = (int64_t)n * tiles_x * tiles_y;
  const unsigned grid = (unsigned)(tiles < g_num_cus ? tiles : g_num_cus);  // persistent: one per CU
  if (res)
    hipLaunchKernelGGL(conv3x3_c64_bf16_kernel<true>, dim3(grid), dim3(512), 0, as_stream(stream), x, w16, scale,
                       shift, y, ldx, ldy, res, ldr, n, h, w, tiles_x, tiles_y, act);
  else
    hipLaunchKernelGGL(conv3x3_c64_bf16_kernel<false>, dim3(grid), dim3(512), 0, as_stream(stream), x, w16, scale,
                       shift, y, ldx, ldy, res, ldr, n, h, w, tiles_x, tiles_y, act);
  return check_launch("sp_conv3x3_c64_bf16");
}
