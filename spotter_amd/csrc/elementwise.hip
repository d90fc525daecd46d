// Memory-bound helpers of the RT-DETRv2 path (NHWC, fp32, float4-vectorised).
//   maxpool 3×3/2 (RN:88), avgpool 2×2 ceil (RN:150/202), nearest ×2 upsample
//   into a concat slice (M2:1192-1193), LayerNorm (nn.LayerNorm), row gather
//   (M2:1601-1617), reference-box init / refinement (M2:616, M2:636-639).
#include "common.h"

namespace sp {
namespace {

__device__ __forceinline__ int64_t grid_stride() { return (int64_t)gridDim.x * blockDim.x; }
__device__ __forceinline__ int64_t gtid() { return (int64_t)blockIdx.x * blockDim.x + threadIdx.x; }

inline unsigned grid_for(int64_t work, int block = 256) {
  int64_t g = (work + block - 1) / block;
  if (g > 256 * 16) g = 256 * 16;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// c4 = channels / 4. Chunks of MP_ROWS output rows of one image over blockIdx.y (strided past 65535), wo·c4 float4s
// across blockIdx.x × threads, 32-bit index math (the grid-stride form's 64-bit divisions dominated at 4.7 TB/s).
// A thread walks its chunk's rows top-down: the 3-tap row maximum of input row 2·oy + 1 is kept for output row
// oy + 1, so each output reads 6 input float4s instead of 9. max is exact, so any order gives the same bits.
// rpc (rows per chunk) = MP_ROWS on large maps (1.04-1.05x at C2 / C3, profiles/r5/pool/rowwalk_*), 1 where
// the chunks would leave the grid short of workgroups (bs1: 0.75x with 4).
constexpr int MP_ROWS = 4;
inline int maxpool_rows_per_chunk(int n, int ho, int gx) {
  return (int64_t)n * ho * gx >= 16384 ? MP_ROWS : 1;  // >= 16 workgroups per CU with the chunks
}

__global__ __launch_bounds__(256) void maxpool3s2_kernel(const float4* __restrict__ x, float4* __restrict__ y,
                                                         int n, int h, int w, int c4, int ho, int wo, int64_t ldy4,
                                                         int rpc) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= wo * c4) return;
  const int ox = j / c4, cc = j - ox * c4;
  const int chunks = (ho + rpc - 1) / rpc;
  const float4 ninf = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
  auto hmax = [&](int b, int iy) {  // max over the 3 taps of input row iy (-inf outside the map)
    float4 m = ninf;
    if ((unsigned)iy >= (unsigned)h) return m;
    const float4* xr = x + ((int64_t)b * h + iy) * w * c4 + cc;
    SP_BCHECK((int64_t)b * h + iy, (int64_t)n * h);
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int ix = ox * 2 - 1 + dx;
      if ((unsigned)ix >= (unsigned)w) continue;
      const float4 v = xr[ix * c4];
      m.x = fmaxf(m.x, v.x); m.y = fmaxf(m.y, v.y); m.z = fmaxf(m.z, v.z); m.w = fmaxf(m.w, v.w);
    }
    return m;
  };
  for (int ch = blockIdx.y; ch < n * chunks; ch += gridDim.y) {
    const int b = ch / chunks, oy0 = (ch - b * chunks) * rpc;
    const int oy1 = oy0 + rpc < ho ? oy0 + rpc : ho;
    float4 prev = hmax(b, 2 * oy0 - 1);
    for (int oy = oy0; oy < oy1; ++oy) {
      const float4 r0 = hmax(b, 2 * oy), r1 = hmax(b, 2 * oy + 1);
      float4 m;
      m.x = fmaxf(fmaxf(prev.x, r0.x), r1.x); m.y = fmaxf(fmaxf(prev.y, r0.y), r1.y);
      m.z = fmaxf(fmaxf(prev.z, r0.z), r1.z); m.w = fmaxf(fmaxf(prev.w, r0.w), r1.w);
      SP_BCHECK(((int64_t)b * ho + oy) * wo + ox, (int64_t)n * ho * wo);
      y[(((int64_t)b * ho + oy) * wo + ox) * ldy4 + cc] = m;
      prev = r1;
    }
  }
}

// Same 2-D grid as maxpool3s2_kernel: output rows over blockIdx.y, wo·c4 float4s over x.
__global__ __launch_bounds__(256) void avgpool2_kernel(const float4* __restrict__ x, float4* __restrict__ y,
                                                       int n, int h, int w, int c4, int ho, int wo, int64_t ldy4) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= wo * c4) return;
  const int ox = j / c4, cc = j - ox * c4;
  for (int row = blockIdx.y; row < n * ho; row += gridDim.y) {  // row = b * ho + oy
    const int oy = row % ho, b = row / ho;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int cnt = 0;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      const int iy = oy * 2 + dy;
      if (iy >= h) continue;
      const float4* xr = x + ((int64_t)b * h + iy) * w * c4 + cc;
      SP_BCHECK((int64_t)b * h + iy, (int64_t)n * h);
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int ix = ox * 2 + dx;
        if (ix >= w) continue;
        const float4 v = xr[ix * c4];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        ++cnt;
      }
    }
    const float inv = (float)cnt;
    y[((int64_t)row * wo + ox) * ldy4 + cc] = make_float4(s.x / inv, s.y / inv, s.z / inv, s.w / inv);
  }
}

// bf16 rows (the bf16 variant's backbone maps, ABI v10): 8 channels (16 bytes) per thread, same 2-D grid.
__device__ __forceinline__ void unpack8(const uint4 u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __builtin_bit_cast(float, w[i] << 16);
    f[2 * i + 1] = __builtin_bit_cast(float, w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b2));
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pk_bf16(f[0], f[1]), pk_bf16(f[2], f[3]), pk_bf16(f[4], f[5]), pk_bf16(f[6], f[7]));
}

__global__ __launch_bounds__(256) void maxpool3s2_bf16_kernel(const uint4* __restrict__ x, uint4* __restrict__ y,
                                                              int n, int h, int w, int c8, int ho, int wo,
                                                              int64_t ldy8, int rpc) {
  // the fp32 kernel's row walk (rpc output rows per chunk, one 3-tap row maximum carried between rows)
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= wo * c8) return;
  const int ox = j / c8, cc = j - ox * c8;
  const int chunks = (ho + rpc - 1) / rpc;
  auto hmax = [&](int b, int iy, float* m) {
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
    if ((unsigned)iy >= (unsigned)h) return;
    const uint4* xr = x + ((int64_t)b * h + iy) * w * c8 + cc;
    SP_BCHECK((int64_t)b * h + iy, (int64_t)n * h);
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int ix = ox * 2 - 1 + dx;
      if ((unsigned)ix >= (unsigned)w) continue;
      float f[8];
      unpack8(xr[ix * c8], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], f[e]);
    }
  };
  for (int ch = blockIdx.y; ch < n * chunks; ch += gridDim.y) {
    const int b = ch / chunks, oy0 = (ch - b * chunks) * rpc;
    const int oy1 = oy0 + rpc < ho ? oy0 + rpc : ho;
    float prev[8], r0[8], r1[8];
    hmax(b, 2 * oy0 - 1, prev);
    for (int oy = oy0; oy < oy1; ++oy) {
      hmax(b, 2 * oy, r0);
      hmax(b, 2 * oy + 1, r1);
      float m[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        m[e] = fmaxf(fmaxf(prev[e], r0[e]), r1[e]);
        prev[e] = r1[e];
      }
      y[(((int64_t)b * ho + oy) * wo + ox) * ldy8 + cc] = pack8(m);  // exact: every max is a bf16 value
    }
  }
}

__global__ __launch_bounds__(256) void avgpool2_bf16_kernel(const uint4* __restrict__ x, uint4* __restrict__ y,
                                                            int n, int h, int w, int c8, int ho, int wo,
                                                            int64_t ldy8) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= wo * c8) return;
  const int ox = j / c8, cc = j - ox * c8;
  for (int row = blockIdx.y; row < n * ho; row += gridDim.y) {
    const int oy = row % ho, b = row / ho;
    float s[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = 0.f;
    int cnt = 0;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      const int iy = oy * 2 + dy;
      if (iy >= h) continue;
      const uint4* xr = x + ((int64_t)b * h + iy) * w * c8 + cc;
      SP_BCHECK((int64_t)b * h + iy, (int64_t)n * h);
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int ix = ox * 2 + dx;
        if (ix >= w) continue;
        float f[8];
        unpack8(xr[ix * c8], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += f[e];
        ++cnt;
      }
    }
    const float inv = (float)cnt;
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] /= inv;
    y[((int64_t)row * wo + ox) * ldy8 + cc] = pack8(s);
  }
}

// One thread per input float4: read once, stored to its 2×2 output block. Input rows over blockIdx.y (strided),
// the row's w·c4 float4s over x, 32-bit index math (the previous form decomposed every output float4's flat index
// with four 64-bit divisions and re-read each input float4 four times: 2.9 TB/s at C2).
__global__ __launch_bounds__(256) void upsample2_kernel(const float4* __restrict__ x, int64_t ldx4,
                                                        float4* __restrict__ y, int64_t ldy4, int n, int h, int w,
                                                        int c4) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= w * c4) return;
  const int ix = j / c4, cc = j - ix * c4;
  const int wo = 2 * w;
  for (int row = blockIdx.y; row < n * h; row += gridDim.y) {  // row = b * h + iy
    const int b = row / h, iy = row - b * h;
    SP_BCHECK(row, (int64_t)n * h);
    SP_BCHECK(((int64_t)b * 2 * h + 2 * iy + 1) * wo + 2 * ix + 1, (int64_t)n * 4 * h * w);
    const float4 v = x[((int64_t)row * w + ix) * ldx4 + cc];
    float4* y0 = y + (((int64_t)b * 2 * h + 2 * iy) * wo + 2 * ix) * ldy4 + cc;
    float4* y1 = y0 + (int64_t)wo * ldy4;
    y0[0] = v;
    y0[ldy4] = v;
    y1[0] = v;
    y1[ldy4] = v;
  }
}

// One wave per row; d <= 1024 (16 floats per lane).
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int64_t ldx,
                                                         const float* __restrict__ g,
                                                         const float* __restrict__ b,
                                                         float* __restrict__ y, int64_t ldy,
                                                         int rows, int d, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * ldx;
  float v[16];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    int c = lane + 64 * i;
    v[i] = c < d ? xr[c] : 0.f;
    s += v[i];
  }
  const float mean = wave_sum(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    int c = lane + 64 * i;
    float t = c < d ? v[i] - mean : 0.f;
    q += t * t;
  }
  const float var = wave_sum(q) / (float)d;
  const float rstd = 1.0f / sqrtf(var + eps);
  float* yr = y + row * ldy;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    int c = lane + 64 * i;
    if (c < d) yr[c] = (v[i] - mean) * rstd * g[c] + b[c];
  }
}

// float4 variant (d, ldx, ldy multiples of 4, 16-byte aligned rows): one wave per row, up to 4 float4
// per lane (d <= 1024). Same two-pass mean / variance as above, 4x fewer load / store instructions.
__global__ __launch_bounds__(256) void layernorm4_kernel(const float* __restrict__ x, int64_t ldx,
                                                          const float* __restrict__ g,
                                                          const float* __restrict__ b,
                                                          float* __restrict__ y, int64_t ldy,
                                                          int rows, int d, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int d4 = d >> 2;
  const float4* xr = reinterpret_cast<const float4*>(x + row * ldx);
  float4 v[4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < d4 ? xr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = wave_sum(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i;
    if (c < d4) {
      const float a0 = v[i].x - mean, a1 = v[i].y - mean, a2 = v[i].z - mean, a3 = v[i].w - mean;
      q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
    }
  }
  const float var = wave_sum(q) / (float)d;
  const float rstd = 1.0f / sqrtf(var + eps);
  float4* yr = reinterpret_cast<float4*>(y + row * ldy);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const float4* b4 = reinterpret_cast<const float4*>(b);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i;
    if (c < d4) {
      const float4 gg = g4[c], bb = b4[c];
      yr[c] = make_float4((v[i].x - mean) * rstd * gg.x + bb.x, (v[i].y - mean) * rstd * gg.y + bb.y,
                          (v[i].z - mean) * rstd * gg.z + bb.z, (v[i].w - mean) * rstd * gg.w + bb.w);
    }
  }
}

// d = 256 (every LayerNorm of the R18vd / R101vd decoders and of the R18vd AIFI): four rows per wave, a 16-lane
// group per row holding four float4 each, the two reductions over the group (4 xor steps), gamma / beta loaded
// before the row so their latency overlaps it. The one-row-per-wave form above ran these at 1.5-1.7 TB/s
// (76800 decoder rows at C3: 94 µs per launch): a single dependent load → reduce → load → store chain per wave.
__device__ __forceinline__ float group16_sum(float v) {
  v += __shfl_xor(v, 8);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 1);
  return v;
}

// y16 (instead of y): the normalised row rounded RNE to bf16 (sp_layernorm_bf16), for a consumer that rounds its
// operand to bf16 anyway (the bf16 variant's encoder score head). One instantiation for both stores, so the row
// arithmetic is compiled once: the bf16 rows are exactly the fp32 rows rounded.
__global__ __launch_bounds__(256) void layernorm256_kernel(const float* __restrict__ x, int64_t ldx,
                                                           const float* __restrict__ g,
                                                           const float* __restrict__ b,
                                                           float* __restrict__ y, uint16_t* __restrict__ y16,
                                                           int64_t ldy, int rows, float eps) {
  const int lane = threadIdx.x & 63, l16 = lane & 15;
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + (lane >> 4);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const float4* b4 = reinterpret_cast<const float4*>(b);
  float4 gg[4], bb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    gg[i] = g4[l16 + 16 * i];
    bb[i] = b4[l16 + 16 * i];
  }
  if (row >= rows) return;  // a 16-lane group shares its row: the whole group leaves together
  const float4* xr = reinterpret_cast<const float4*>(x + row * ldx);
  float4 v[4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = xr[l16 + 16 * i];
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
  const float mean = group16_sum(s) * (1.0f / 256.0f);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a0 = v[i].x - mean, a1 = v[i].y - mean, a2 = v[i].z - mean, a3 = v[i].w - mean;
    q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
  }
  const float var = group16_sum(q) * (1.0f / 256.0f);
  const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 o = make_float4((v[i].x - mean) * rstd * gg[i].x + bb[i].x, (v[i].y - mean) * rstd * gg[i].y + bb[i].y,
                                 (v[i].z - mean) * rstd * gg[i].z + bb[i].z, (v[i].w - mean) * rstd * gg[i].w + bb[i].w);
    if (y16)
      reinterpret_cast<uint2*>(y16 + row * ldy)[l16 + 16 * i] = make_uint2(pk_bf16(o.x, o.y), pk_bf16(o.z, o.w));
    else
      reinterpret_cast<float4*>(y + row * ldy)[l16 + 16 * i] = o;
  }
}

__global__ void gather_rows_kernel(const float* __restrict__ src, int64_t ld_src, int src_rows,
                                   const int32_t* __restrict__ idx, int k, int batch, int d,
                                   float* __restrict__ dst, int64_t ld_dst) {
  const int64_t total = (int64_t)batch * k * d;
  for (int64_t i = gtid(); i < total; i += grid_stride()) {
    int c = (int)(i % d);
    int64_t r = i / d;  // b*k + j
    int b = (int)(r / k);
    SP_BCHECK(idx[r], src_rows);  // a selected row (top-k index) inside its image's rows
    int64_t s = (int64_t)b * src_rows + idx[r];
    dst[r * ld_dst + c] = src[s * ld_src + c];
  }
}

// y = a + b over `rows` rows of 8·c8 columns (fp32 in), stored as fp32 rows or rounded RNE to bf16 rows: the
// attention input q = k = h + pos (M2:395-404 / 409-423) materialised once so that the query / offset
// projections take their A operand by LDS-DMA. The bf16 form is the operand the bf16-mode GEMM would have
// rounded in its own loader (v_cvt_pk_bf16_f32 of the same fp32 sum), so the products are unchanged.
__global__ __launch_bounds__(256) void add_rows_kernel(const float* __restrict__ a, int64_t lda,
                                                       const float* __restrict__ b, int64_t ldb,
                                                       float* __restrict__ y, uint16_t* __restrict__ y16,
                                                       int64_t ldy, int rows, int c8) {
  const int64_t total = (int64_t)rows * c8;
  for (int64_t i = gtid(); i < total; i += grid_stride()) {
    const int64_t r = i / c8;
    const int q = (int)(i - r * c8) * 8;
    SP_BCHECK(q + 7, lda < ldb ? lda : ldb);
    SP_BCHECK(q + 7, ldy);
    const float4* pa = reinterpret_cast<const float4*>(a + r * lda + q);
    const float4* pb = reinterpret_cast<const float4*>(b + r * ldb + q);
    const float4 a0 = pa[0], a1 = pa[1], b0 = pb[0], b1 = pb[1];
    const float f[8] = {a0.x + b0.x, a0.y + b0.y, a0.z + b0.z, a0.w + b0.w,
                        a1.x + b1.x, a1.y + b1.y, a1.z + b1.z, a1.w + b1.w};
    if (y16) {
      *reinterpret_cast<uint4*>(y16 + r * ldy + q) = pack8(f);
    } else {
      float4* py = reinterpret_cast<float4*>(y + r * ldy + q);
      py[0] = make_float4(f[0], f[1], f[2], f[3]);
      py[1] = make_float4(f[4], f[5], f[6], f[7]);
    }
  }
}

__global__ void ref_init_kernel(const float* __restrict__ delta, int64_t ld, const float* __restrict__ anchors,
                                const int32_t* __restrict__ idx, int batch, int k,
                                float* __restrict__ ref) {
  const int64_t total = (int64_t)batch * k * 4;
  for (int64_t i = gtid(); i < total; i += grid_stride()) {
    int c = (int)(i & 3);
    int64_t r = i >> 2;
    SP_BCHECK(idx[r], 0x7fffffff);  // (the anchor count is not passed: at least not negative)
    float u = delta[r * ld + c] + anchors[(int64_t)idx[r] * 4 + c];
    ref[i] = sigmoidf_(u);
  }
}

__global__ void box_refine_kernel(const float* __restrict__ delta, int64_t ld, float* __restrict__ ref,
                                  int rows) {
  const int64_t total = (int64_t)rows * 4;
  for (int64_t i = gtid(); i < total; i += grid_stride()) {
    int c = (int)(i & 3);
    int64_t r = i >> 2;
    float x = fminf(fmaxf(ref[i], 0.f), 1.f);
    float x1 = fmaxf(x, 1e-5f);
    float x2 = fmaxf(1.f - x, 1e-5f);
    float inv = logf(x1 / x2);
    ref[i] = sigmoidf_(delta[r * ld + c] + inv);
  }
}

// NCHW pixel_values (the processor contract, IPP:461-462) → NHWC for the stem conv.
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, float* __restrict__ y, int n, int c, int hw) {
  const int64_t total = (int64_t)n * c * hw;
  for (int64_t i = gtid(); i < total; i += grid_stride()) {
    int cc = (int)(i % c);
    int64_t p = i / c;
    int b = (int)(p / hw);
    int s = (int)(p - (int64_t)b * hw);
    y[i] = x[((int64_t)b * c + cc) * hw + s];
  }
}

}  // namespace
}  // namespace sp

using namespace sp;

extern "C" int sp_nchw_to_nhwc(const float* x, float* y, int n, int c, int h, int w, void* stream) {
  SP_ARG_CHECK(x && y && n > 0 && c > 0 && h > 0 && w > 0, "sp_nchw_to_nhwc: bad args");
  int64_t work = (int64_t)n * c * h * w;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), x, y, n, c,
                     h * w);
  return check_launch("sp_nchw_to_nhwc");
}

extern "C" int sp_maxpool3x3s2(const float* x, float* y, int64_t ldy, int n, int h, int w, int c, void* stream) {
  SP_ARG_CHECK(x && y && n > 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0 && ldy >= c && ldy % 4 == 0 &&
                   ((uintptr_t)y & 15) == 0,
               "sp_maxpool3x3s2: bad args");
  int ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  SP_ARG_CHECK((int64_t)n * ho < (1 << 30) && (int64_t)wo * (c / 4) < (1 << 30), "sp_maxpool3x3s2: size out of range");
  const int gx = (wo * (c / 4) + 255) / 256;
  const int rpc = maxpool_rows_per_chunk(n, ho, gx);
  const int64_t rows = (int64_t)n * ((ho + rpc - 1) / rpc);
  const int gy = rows < 65535 ? (int)rows : 65535;
  hipLaunchKernelGGL(maxpool3s2_kernel, dim3(gx, gy), dim3(256), 0, as_stream(stream),
                     (const float4*)x, (float4*)y, n, h, w, c / 4, ho, wo, ldy / 4, rpc);
  return check_launch("sp_maxpool3x3s2");
}

extern "C" int sp_avgpool2x2_ceil(const float* x, float* y, int64_t ldy, int n, int h, int w, int c,
                                  void* stream) {
  SP_ARG_CHECK(x && y && n > 0 && h > 0 && w > 0 && c > 0 && c % 4 == 0 && ldy >= c && ldy % 4 == 0 &&
                   ((uintptr_t)y & 15) == 0,
               "sp_avgpool2x2_ceil: bad args");
  int ho = (h + 1) / 2, wo = (w + 1) / 2;
  SP_ARG_CHECK((int64_t)n * ho < (1 << 30) && (int64_t)wo * (c / 4) < (1 << 30), "sp_avgpool2x2_ceil: size out of range");
  const int gy = n * ho < 65535 ? n * ho : 65535;
  hipLaunchKernelGGL(avgpool2_kernel, dim3((wo * (c / 4) + 255) / 256, gy), dim3(256), 0, as_stream(stream),
                     (const float4*)x, (float4*)y, n, h, w, c / 4, ho, wo, ldy / 4);
  return check_launch("sp_avgpool2x2_ceil");
}

extern "C" int sp_maxpool3x3s2_bf16(const uint16_t* x, uint16_t* y, int64_t ldy, int n, int h, int w, int c,
                                    void* stream) {
  SP_ARG_CHECK(x && y && n > 0 && h > 0 && w > 0 && c > 0 && c % 8 == 0 && ldy >= c && ldy % 8 == 0 &&
                   ((uintptr_t)y & 15) == 0 && ((uintptr_t)x & 15) == 0,
               "sp_maxpool3x3s2_bf16: bad args");
  int ho = (h - 1) / 2 + 1, wo = (w - 1) / 2 + 1;
  SP_ARG_CHECK((int64_t)n * ho < (1 << 30) && (int64_t)wo * (c / 8) < (1 << 30), "sp_maxpool3x3s2_bf16: size out of range");
  const int gx = (wo * (c / 8) + 255) / 256;
  const int rpc = maxpool_rows_per_chunk(n, ho, gx);
  const int64_t rows = (int64_t)n * ((ho + rpc - 1) / rpc);
  const int gy = rows < 65535 ? (int)rows : 65535;
  hipLaunchKernelGGL(maxpool3s2_bf16_kernel, dim3(gx, gy), dim3(256), 0, as_stream(stream),
                     (const uint4*)x, (uint4*)y, n, h, w, c / 8, ho, wo, ldy / 8, rpc);
  return check_launch("sp_maxpool3x3s2_bf16");
}

extern "C" int sp_avgpool2x2_ceil_bf16(const uint16_t* x, uint16_t* y, int64_t ldy, int n, int h, int w, int c,
                                       void* stream) {
  SP_ARG_CHECK(x && y && n > 0 && h > 0 && w > 0 && c > 0 && c % 8 == 0 && ldy >= c && ldy % 8 == 0 &&
                   ((uintptr_t)y & 15) == 0 && ((uintptr_t)x & 15) == 0,
               "sp_avgpool2x2_ceil_bf16: bad args");
  int ho = (h + 1) / 2, wo = (w + 1) / 2;
  SP_ARG_CHECK((int64_t)n * ho < (1 << 30) && (int64_t)wo * (c / 8) < (1 << 30), "sp_avgpool2x2_ceil_bf16: size out of range");
  const int gy = n * ho < 65535 ? n * ho : 65535;
  hipLaunchKernelGGL(avgpool2_bf16_kernel, dim3((wo * (c / 8) + 255) / 256, gy), dim3(256), 0, as_stream(stream),
                     (const uint4*)x, (uint4*)y, n, h, w, c / 8, ho, wo, ldy / 8);
  return check_launch("sp_avgpool2x2_ceil_bf16");
}

extern "C" int sp_upsample2x_nearest(const float* x, int64_t ldx, float* y, int64_t ldy, int n, int h,
                                     int w, int c, void* stream) {
  SP_ARG_CHECK(x && y && n > 0 && c % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0, "sp_upsample2x_nearest: bad args");
  SP_ARG_CHECK(h > 0 && w > 0 && (int64_t)n * h < (1 << 30) && (int64_t)w * (c / 4) < (1 << 30) &&
                   ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0,
               "sp_upsample2x_nearest: size out of range or unaligned rows");
  const int gy = n * h < 65535 ? n * h : 65535;
  hipLaunchKernelGGL(upsample2_kernel, dim3((w * (c / 4) + 255) / 256, gy), dim3(256), 0, as_stream(stream),
                     (const float4*)x, ldx / 4, (float4*)y, ldy / 4, n, h, w, c / 4);
  return check_launch("sp_upsample2x_nearest");
}

extern "C" int sp_layernorm(const float* x, int64_t ldx, const float* gamma, const float* beta, float* y,
                            int64_t ldy, int rows, int d, float eps, void* stream) {
  SP_ARG_CHECK(x && gamma && beta && y && rows > 0 && d > 0 && d <= 1024, "sp_layernorm: bad args");
  const bool vec = d % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 &&
                  (((uintptr_t)x | (uintptr_t)y | (uintptr_t)gamma | (uintptr_t)beta) & 15) == 0;
  if (vec && d == 256)
    hipLaunchKernelGGL(layernorm256_kernel, dim3((rows + 15) / 16), dim3(256), 0, as_stream(stream), x, ldx, gamma,
                       beta, y, nullptr, ldy, rows, eps);
  else
    hipLaunchKernelGGL(vec ? layernorm4_kernel : layernorm_kernel, dim3((rows + 3) / 4), dim3(256), 0,
                       as_stream(stream), x, ldx, gamma, beta, y, ldy, rows, d, eps);
  return check_launch("sp_layernorm");
}

extern "C" int sp_layernorm_bf16(const float* x, int64_t ldx, const float* gamma, const float* beta, uint16_t* y,
                                 int64_t ldy, int rows, int d, float eps, void* stream) {
  SP_ARG_CHECK(x && gamma && beta && y && rows > 0 && d == 256 && ldx % 4 == 0 && ldy % 4 == 0 &&
                   (((uintptr_t)x | (uintptr_t)gamma | (uintptr_t)beta) & 15) == 0 && ((uintptr_t)y & 7) == 0,
               "sp_layernorm_bf16: d = 256, ldx / ldy %% 4, 16-byte aligned fp32 rows, 8-byte aligned bf16 rows");
  hipLaunchKernelGGL(layernorm256_kernel, dim3((rows + 15) / 16), dim3(256), 0, as_stream(stream), x, ldx, gamma,
                     beta, nullptr, y, ldy, rows, eps);
  return check_launch("sp_layernorm_bf16");
}

extern "C" int sp_gather_rows(const float* src, int64_t ld_src, int src_rows, const int32_t* idx, int k,
                              int batch, int d, float* dst, int64_t ld_dst, void* stream) {
  SP_ARG_CHECK(src && idx && dst && k > 0 && batch > 0 && d > 0, "sp_gather_rows: bad args");
  int64_t work = (int64_t)batch * k * d;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(work)), dim3(256), 0, as_stream(stream), src,
                     ld_src, src_rows, idx, k, batch, d, dst, ld_dst);
  return check_launch("sp_gather_rows");
}

extern "C" int sp_add_rows(const float* a, int64_t lda, const float* b, int64_t ldb, float* y, uint16_t* y_bf16,
                           int64_t ldy, int rows, int cols, void* stream) {
  SP_ARG_CHECK(a && b && (y != nullptr) != (y_bf16 != nullptr) && rows > 0 && cols > 0,
               "sp_add_rows: bad args (exactly one of y / y_bf16)");
  const uintptr_t al = (uintptr_t)a | (uintptr_t)b | (uintptr_t)(y ? (const void*)y : (const void*)y_bf16);
  SP_ARG_CHECK(cols % 8 == 0 && lda % 4 == 0 && ldb % 4 == 0 && ldy % 8 == 0 && lda >= cols && ldb >= cols &&
                   ldy >= cols && (al & 15) == 0,
               "sp_add_rows: cols %% 8, lda / ldb %% 4, ldy %% 8 and 16-byte aligned rows required");
  hipLaunchKernelGGL(add_rows_kernel, dim3(grid_for((int64_t)rows * (cols / 8))), dim3(256), 0, as_stream(stream),
                     a, lda, b, ldb, y, y_bf16, ldy, rows, cols / 8);
  return check_launch("sp_add_rows");
}

extern "C" int sp_ref_init(const float* delta, int64_t ld_delta, const float* anchors, const int32_t* idx,
                           int batch, int k, float* ref, void* stream) {
  SP_ARG_CHECK(delta && anchors && idx && ref && batch > 0 && k > 0, "sp_ref_init: bad args");
  hipLaunchKernelGGL(ref_init_kernel, dim3(grid_for((int64_t)batch * k * 4)), dim3(256), 0,
                     as_stream(stream), delta, ld_delta, anchors, idx, batch, k, ref);
  return check_launch("sp_ref_init");
}

extern "C" int sp_box_refine(const float* delta, int64_t ld_delta, float* ref, int rows, void* stream) {
  SP_ARG_CHECK(delta && ref && rows > 0, "sp_box_refine: bad args");
  hipLaunchKernelGGL(box_refine_kernel, dim3(grid_for((int64_t)rows * 4)), dim3(256), 0,
                     as_stream(stream), delta, ld_delta, ref, rows);
  return check_launch("sp_box_refine");
}
