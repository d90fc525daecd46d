// JPEG decode in front of A1 (serve.py:96-97: Image.open(BytesIO(..)).convert("RGB"), which Pillow runs
// through libjpeg-turbo). The entropy decode is a serial bit stream and stays on the host (C++ below); the
// per-pixel work runs on the GPU: dequantisation + the ISLOW integer IDCT per 8x8 block (jidctint.c), then
// "fancy" triangle upsampling of the chroma planes (jdsample.c h2v1 / h2v2 / h1v2_fancy_upsample) with the
// edge-row replication of the main controller's context rows (jdmainct.c), then the integer YCbCr→RGB
// tables (jdcolor.c) — the same integer arithmetic, so the pixels are Pillow's, bit for bit.
// libjpeg-turbo is a dependency of Pillow (absent from /root/reference); its published algorithms are
// restated here and in oracle/jpeg_np.py, and tests/test_jpeg.py pins both against Pillow's own decode.
#include <cstdint>
#include <vector>

#include "common.h"

#include "jpeg_host.h"

namespace sp {
namespace {
using namespace jpeg_host;

// ------------------------------------------------------------------------------------------------ device
// jidctint.c jpeg_idct_islow constants (CONST_BITS 13, PASS1_BITS 2)
constexpr int kCB = 13, kP1 = 2;
constexpr int F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373, F1_175 = 9633,
              F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819, F2_562 = 20995, F3_072 = 25172;

// The 1-D ISLOW butterfly on 8 values in (pass 1: dequantised coefficients; pass 2: the workspace row),
// out[i] = (value + rounding) >> shift, exactly the jidctint.c sequence of products and sums.
__device__ __forceinline__ void islow_1d(const int64_t (&in)[8], int shift, int64_t (&out)[8]) {
  int64_t z2 = in[2], z3 = in[6];
  int64_t z1 = (z2 + z3) * F0_541;
  const int64_t tmp2 = z1 + z3 * -F1_847;
  const int64_t tmp3 = z1 + z2 * F0_765;
  z2 = in[0];
  z3 = in[4];
  const int64_t t0 = (z2 + z3) * (1 << kCB);
  const int64_t t1 = (z2 - z3) * (1 << kCB);
  const int64_t tmp10 = t0 + tmp3, tmp13 = t0 - tmp3, tmp11 = t1 + tmp2, tmp12 = t1 - tmp2;
  int64_t o0 = in[7], o1 = in[5], o2 = in[3], o3 = in[1];
  z1 = o0 + o3;
  z2 = o1 + o2;
  z3 = o0 + o2;
  int64_t z4 = o1 + o3;
  const int64_t z5 = (z3 + z4) * F1_175;
  o0 *= F0_298;
  o1 *= F2_053;
  o2 *= F3_072;
  o3 *= F1_501;
  z1 *= -F0_899;
  z2 *= -F2_562;
  z3 *= -F1_961;
  z4 *= -F0_390;
  z3 += z5;
  z4 += z5;
  o0 += z1 + z3;
  o1 += z2 + z4;
  o2 += z2 + z3;
  o3 += z1 + z4;
  const int64_t rnd = (int64_t)1 << (shift - 1);
  out[0] = (tmp10 + o3 + rnd) >> shift;
  out[7] = (tmp10 - o3 + rnd) >> shift;
  out[1] = (tmp11 + o2 + rnd) >> shift;
  out[6] = (tmp11 - o2 + rnd) >> shift;
  out[2] = (tmp12 + o1 + rnd) >> shift;
  out[5] = (tmp12 - o1 + rnd) >> shift;
  out[3] = (tmp13 + o0 + rnd) >> shift;
  out[4] = (tmp13 - o0 + rnd) >> shift;
}

// IDCT_range_limit: the & RANGE_MASK (1023) wrap, then clamp of value + 128 to [0, 255] (jdmaster.c
// prepare_range_limit_table)
__device__ __forceinline__ uint8_t idct_limit(int64_t x) {
  int v = (int)(x & 1023);
  v = v >= 512 ? v - 1024 : v;
  v += 128;
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// The envelope in which this (jidctint.c) arithmetic and libjpeg-turbo's SIMD IDCT, which Pillow runs on x86,
// give the same samples: dequantised coefficients and pass-1 values that fit 15-bit signed arithmetic with a
// pairwise sum to spare (the SIMD code multiplies and adds 16-bit lanes and packs pass 1 with saturation), and
// pass-2 values inside [-512, 511] (where the C range-limit table's & 1023 wrap and the SIMD saturating packs
// both reduce to clamp(x + 128)). Well-formed files stay far inside it; a block outside it (corrupt or
// crafted data) sets *status, and the caller gives that file to Pillow.
constexpr int64_t kEnv16 = (1 << 14) - 1;

// 8 threads per 8x8 block (thread = column in pass 1, row in pass 2), 32 blocks per workgroup.
__global__ __launch_bounds__(256) void jpeg_idct_kernel(const int16_t* __restrict__ coefs, const sp_jpeg_layout L,
                                                        uint8_t* __restrict__ work, int32_t* __restrict__ status) {
  __shared__ int32_t ws[32][8][9];
  const int lb = threadIdx.x >> 3, t = threadIdx.x & 7;
  const int64_t blk = (int64_t)blockIdx.x * 32 + lb;
  const bool live = blk < L.total_blocks;
  int c = 0;
  if (L.ncomp > 1 && blk >= L.block_off[1]) c = 1;
  if (L.ncomp > 2 && blk >= L.block_off[2]) c = 2;
  bool outside = false;
  if (live) {
    const int16_t* in = coefs + blk * 64;
    int64_t col[8], out[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      col[r] = (int64_t)in[r * 8 + t] * L.quant[c][r * 8 + t];
      outside |= col[r] > kEnv16 || col[r] < -kEnv16;
    }
    islow_1d(col, kCB - kP1, out);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      ws[lb][r][t] = (int32_t)out[r];
      outside |= out[r] > kEnv16 || out[r] < -kEnv16;
    }
  }
  __syncthreads();
  if (!live) return;
  int64_t row[8], out[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) row[i] = ws[lb][t][i];
  islow_1d(row, kCB + kP1 + 3, out);
#pragma unroll
  for (int i = 0; i < 8; ++i) outside |= out[i] > 511 || out[i] < -512;
  if (outside && status) *status = 1;
  const int64_t local = blk - L.block_off[c];
  const int by = (int)(local / L.bw[c]), bx = (int)(local - (int64_t)by * L.bw[c]);
  const int64_t stride = (int64_t)L.bw[c] * 8;
  SP_BCHECK(by, L.bh[c]);  // the block's position inside its component's block grid
  SP_BCHECK(L.plane_off[c] + ((int64_t)by * 8 + t) * stride + (int64_t)bx * 8 + 7, L.plane_bytes);
  uint8_t* dst = work + L.plane_off[c] + ((int64_t)by * 8 + t) * stride + (int64_t)bx * 8;
  uint32_t w0 = 0, w1 = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w0 |= (uint32_t)idct_limit(out[i]) << (8 * i);
    w1 |= (uint32_t)idct_limit(out[i + 4]) << (8 * i);
  }
  *reinterpret_cast<uint2*>(dst) = make_uint2(w0, w1);
}

// One chroma sample at output (x, y): jdsample.c fancy upsampling (triangle filter 3/4 nearer + 1/4 further
// in each upsampled direction), rows past the component's edge replicating its first / last row as the
// main controller's context rows do; box replication where libjpeg-turbo picks it (downsampled width <= 2
// for the horizontal-doubling forms).
__device__ __forceinline__ int chroma_at(const uint8_t* pl, int64_t stride, int rh, int rv, int dw, int dh, int x,
                                         int y) {
  if (rh == 1 && rv == 1) return pl[(int64_t)y * stride + x];
  const int xc = rh == 2 ? x >> 1 : x, yc = rv == 2 ? y >> 1 : y;
  if (rh == 2 && dw <= 2) return pl[(int64_t)yc * stride + xc];  // h2v1_upsample / h2v2_upsample
  if (rh == 2 && rv == 1) {  // h2v1_fancy_upsample
    const uint8_t* r = pl + (int64_t)yc * stride;
    const int in = r[xc];
    if ((x & 1) == 0) return xc == 0 ? in : (in * 3 + r[xc - 1] + 1) >> 2;
    return xc == dw - 1 ? in : (in * 3 + r[xc + 1] + 2) >> 2;
  }
  // vertical doubling: the nearer row yc and the further row above (even y) or below (odd y)
  const int yn = (y & 1) ? (yc + 1 < dh ? yc + 1 : dh - 1) : (yc > 0 ? yc - 1 : 0);
  const uint8_t* r0 = pl + (int64_t)yc * stride;
  const uint8_t* r1 = pl + (int64_t)yn * stride;
  if (rh == 1) return (r0[x] * 3 + r1[x] + ((y & 1) ? 2 : 1)) >> 2;  // h1v2_fancy_upsample
  // h2v2_fancy_upsample: column sums 3·nearer row + further row, then 3/4 · 1/4 across columns
  const int cs = r0[xc] * 3 + r1[xc];
  if ((x & 1) == 0) {
    if (xc == 0) return (cs * 4 + 8) >> 4;
    return (cs * 3 + r0[xc - 1] * 3 + r1[xc - 1] + 8) >> 4;
  }
  if (xc == dw - 1) return (cs * 4 + 7) >> 4;
  return (cs * 3 + r0[xc + 1] * 3 + r1[xc + 1] + 7) >> 4;
}

__device__ __forceinline__ uint8_t clamp8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// One thread per output pixel: luma from its plane, chroma upsampled, jdcolor.c ycc_rgb_convert (SCALEBITS 16
// fixed point: Cr→R 1.40200, Cb→B 1.77200, G = y + ((−0.34414·Cb + ½ − 0.71414·Cr) >> 16)).
__global__ __launch_bounds__(256) void jpeg_color_kernel(const sp_jpeg_layout L, const uint8_t* __restrict__ work,
                                                         uint8_t* __restrict__ rgb, int64_t rgb_stride) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)L.width * L.height) return;
  const int y = (int)(i / L.width), x = (int)(i - (int64_t)y * L.width);
  uint8_t* o = rgb + (int64_t)y * rgb_stride + (int64_t)x * 3;
  SP_BCHECK(L.plane_off[0] + (int64_t)y * L.bw[0] * 8 + x, L.ncomp > 1 ? L.plane_off[1] : L.plane_bytes);
  const int yy = work[L.plane_off[0] + (int64_t)y * L.bw[0] * 8 + x];
  if (L.ncomp == 1) {
    o[0] = o[1] = o[2] = (uint8_t)yy;
    return;
  }
  int cc[2];
#pragma unroll
  for (int k = 1; k < 3; ++k) {
    const int rh = L.max_h / L.h[k], rv = L.max_v / L.v[k];
    const int dw = (int)(((int64_t)L.width * L.h[k] + L.max_h - 1) / L.max_h);
    const int dh = (int)(((int64_t)L.height * L.v[k] + L.max_v - 1) / L.max_v);
    // the rows / columns chroma_at reads: [0, dh) × [0, dw) of a plane bw·8 wide and bh·8 high
    SP_BCHECK((rv == 2 ? y >> 1 : y), (int64_t)L.bh[k] * 8);
    SP_BCHECK((rh == 2 ? x >> 1 : x), dw);
    SP_BCHECK(L.plane_off[k] + ((int64_t)L.bh[k] * 8 - 1) * L.bw[k] * 8 + L.bw[k] * 8 - 1, k == 1 && L.ncomp > 2 ? L.plane_off[2] : L.plane_bytes);
    cc[k - 1] = chroma_at(work + L.plane_off[k], (int64_t)L.bw[k] * 8, rh, rv, dw, dh, x, y);
  }
  if (L.color == 2) {  // RGB components: no conversion
    o[0] = (uint8_t)yy;
    o[1] = (uint8_t)cc[0];
    o[2] = (uint8_t)cc[1];
    return;
  }
  const int cb = cc[0] - 128, cr = cc[1] - 128;
  const int r_off = (91881 * cr + 32768) >> 16;
  const int b_off = (116130 * cb + 32768) >> 16;
  const int g_off = (-22554 * cb + 32768 + -46802 * cr) >> 16;
  o[0] = clamp8(yy + r_off);
  o[1] = clamp8(yy + g_off);
  o[2] = clamp8(yy + b_off);
}

}  // namespace
}  // namespace sp

extern "C" int sp_jpeg_decode_coefs(const uint8_t* data, int64_t len, sp_jpeg_layout* lay, int16_t* coefs,
                                    int64_t coef_elems) {
  using namespace sp;
  SP_ARG_CHECK(data && lay && len > 0, "sp_jpeg_decode_coefs: null args");
  Decoder d{data, len, lay, coefs};
  const int rc = d.run(false);
  if (rc || !coefs) return rc;
  SP_ARG_CHECK(coef_elems >= lay->total_blocks * 64, "sp_jpeg_decode_coefs: coefficient buffer holds %lld < %lld",
               (long long)coef_elems, (long long)(lay->total_blocks * 64));
  Decoder d2{data, len, lay, coefs};
  return d2.run(true);
}

extern "C" int sp_jpeg_to_rgb(const int16_t* coefs, const sp_jpeg_layout* lay, uint8_t* work, int64_t work_bytes,
                              uint8_t* rgb, int64_t rgb_stride, int32_t* status, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(coefs && lay && work && rgb, "sp_jpeg_to_rgb: null args");
  SP_ARG_CHECK(lay->ncomp == 1 || lay->ncomp == 3, "sp_jpeg_to_rgb: ncomp %d", lay->ncomp);
  SP_ARG_CHECK(work_bytes >= lay->plane_bytes, "sp_jpeg_to_rgb: work %lld < %lld bytes", (long long)work_bytes,
               (long long)lay->plane_bytes);
  SP_ARG_CHECK(rgb_stride >= 3LL * lay->width, "sp_jpeg_to_rgb: rgb_stride");
  for (int c = 0; c < lay->ncomp; ++c)
    SP_ARG_CHECK((int64_t)lay->bw[c] * 8 >= ((int64_t)lay->width * lay->h[c] + lay->max_h - 1) / lay->max_h &&
                     (int64_t)lay->bh[c] * 8 >= ((int64_t)lay->height * lay->v[c] + lay->max_v - 1) / lay->max_v &&
                     (reinterpret_cast<uintptr_t>(work + lay->plane_off[c]) & 7) == 0,
                 "sp_jpeg_to_rgb: inconsistent layout");
  hipStream_t s = as_stream(stream);
  const int64_t g1 = (lay->total_blocks + 31) / 32;
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)g1), dim3(256), 0, s, coefs, *lay, work, status);
  int rc = check_launch("sp_jpeg_to_rgb(idct)");
  if (rc) return rc;
  const int64_t px = (int64_t)lay->width * lay->height;
  hipLaunchKernelGGL(jpeg_color_kernel, dim3((unsigned)((px + 255) / 256)), dim3(256), 0, s, *lay, work, rgb,
                     rgb_stride);
  return check_launch("sp_jpeg_to_rgb(color)");
}
