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
