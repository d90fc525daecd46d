// Small fused multi-head self-attention (AIFI: 400 tokens × 8 heads × 48 at
// 640²; decoder: 300 queries × 8 heads × 32). softmax(Q Kᵀ · scale) V with an
// online (running max / sum) softmax corrected once per block of 16 keys, one query
// per lane, K/V tiles of 64 keys broadcast from LDS. Restates eager_attention_forward / sdpa (M2:245-270) as
// called by RTDetrV2SelfAttention (M2:300-336); Q/K/V/O projections run on the
// MFMA GEMM (conv_gemm.hip). ≈1 % of the step's FLOPs, VALU-bound.
#include "common.h"

namespace sp {
namespace {

constexpr int KT = 64;

template <int DH>
__global__ __launch_bounds__(64) void attn_kernel(const float* __restrict__ q, int64_t ldq,
                                                  const float* __restrict__ k, int64_t ldk,
                                                  const float* __restrict__ v, int64_t ldv,
                                                  float* __restrict__ o, int64_t ldo, int n,
                                                  float scale) {
  __shared__ __attribute__((aligned(16))) float Ks[KT * DH];
  __shared__ __attribute__((aligned(16))) float Vs[KT * DH];
  const int lane = threadIdx.x;
  const int b = blockIdx.z;
  const int hh = blockIdx.y;
  const int qi = blockIdx.x * 64 + lane;
  const bool valid = qi < n;
  const int64_t rowbase = (int64_t)b * n;
  float qv[DH], acc[DH];
  const float* qr = q + (rowbase + (valid ? qi : 0)) * ldq + hh * DH;
#pragma unroll
  for (int c = 0; c < DH; c += 4) {
    float4 t = *reinterpret_cast<const float4*>(qr + c);
    qv[c] = t.x; qv[c + 1] = t.y; qv[c + 2] = t.z; qv[c + 3] = t.w;
    acc[c] = acc[c + 1] = acc[c + 2] = acc[c + 3] = 0.f;
  }
  // online softmax per block of SB keys: one running-max correction per block instead of per key
  constexpr int SB = 16;
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < n; k0 += KT) {
    const int nk = min(KT, n - k0);
    __syncthreads();
    for (int idx = lane; idx < nk * (DH / 4); idx += 64) {
      const int r = idx / (DH / 4);
      const int c = (idx - r * (DH / 4)) * 4;
      *reinterpret_cast<float4*>(Ks + r * DH + c) =
          *reinterpret_cast<const float4*>(k + (rowbase + k0 + r) * ldk + hh * DH + c);
      *reinterpret_cast<float4*>(Vs + r * DH + c) =
          *reinterpret_cast<const float4*>(v + (rowbase + k0 + r) * ldv + hh * DH + c);
    }
    __syncthreads();
    for (int j0 = 0; j0 < nk; j0 += SB) {
      float sc[SB];
      float mt = -INFINITY;
#pragma unroll
      for (int jj = 0; jj < SB; ++jj) {
        const float* kr = Ks + (j0 + jj) * DH;
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < DH; c += 4) {
          float4 t = *reinterpret_cast<const float4*>(kr + c);
          s = fmaf(qv[c], t.x, s);
          s = fmaf(qv[c + 1], t.y, s);
          s = fmaf(qv[c + 2], t.z, s);
          s = fmaf(qv[c + 3], t.w, s);
        }
        s *= scale;
        sc[jj] = (j0 + jj < nk) ? s : -INFINITY;
        mt = fmaxf(mt, sc[jj]);
      }
      const float mn = fmaxf(m, mt);
      const float corr = expf(m - mn);  // m = -inf on the first block: corr = 0, acc / l are 0
      l *= corr;
#pragma unroll
      for (int c = 0; c < DH; ++c) acc[c] *= corr;
      m = mn;
#pragma unroll
      for (int jj = 0; jj < SB; ++jj) {
        if (j0 + jj < nk) {  // wave-uniform; rows past nk hold stale LDS
          const float pj = expf(sc[jj] - mn);
          l += pj;
          const float* vr = Vs + (j0 + jj) * DH;
#pragma unroll
          for (int c = 0; c < DH; c += 4) {
            float4 t = *reinterpret_cast<const float4*>(vr + c);
            acc[c] = fmaf(pj, t.x, acc[c]);
            acc[c + 1] = fmaf(pj, t.y, acc[c + 1]);
            acc[c + 2] = fmaf(pj, t.z, acc[c + 2]);
            acc[c + 3] = fmaf(pj, t.w, acc[c + 3]);
          }
        }
      }
    }
  }
  if (!valid) return;
  const float inv = 1.0f / l;
  float* orow = o + (rowbase + qi) * ldo + hh * DH;
#pragma unroll
  for (int c = 0; c < DH; c += 4)
    *reinterpret_cast<float4*>(orow + c) = make_float4(acc[c] * inv, acc[c + 1] * inv, acc[c + 2] * inv, acc[c + 3] * inv);
}

template <int DH>
int launch(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v, int64_t ldv,
           float* o, int64_t ldo, int batch, int n, int heads, float scale, hipStream_t s) {
  dim3 grid((n + 63) / 64, heads, batch);
  hipLaunchKernelGGL((attn_kernel<DH>), grid, dim3(64), 0, s, q, ldq, k, ldk, v, ldv, o, ldo, n, scale);
  return check_launch("sp_attention");
}

}  // namespace
}  // namespace sp

extern "C" int sp_attention(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v,
                            int64_t ldv, float* o, int64_t ldo, int batch, int n, int heads, int dh,
                            float scale, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(q && k && v && o && batch > 0 && n > 0 && heads > 0, "sp_attention: bad args");
  SP_ARG_CHECK(ldq % 4 == 0 && ldk % 4 == 0 && ldv % 4 == 0 && ldo % 4 == 0, "sp_attention: ld % 4");
  hipStream_t s = as_stream(stream);
  switch (dh) {
    case 32: return launch<32>(q, ldq, k, ldk, v, ldv, o, ldo, batch, n, heads, scale, s);
    case 48: return launch<48>(q, ldq, k, ldk, v, ldv, o, ldo, batch, n, heads, scale, s);
    case 64: return launch<64>(q, ldq, k, ldk, v, ldv, o, ldo, batch, n, heads, scale, s);
    default: set_error("sp_attention: head_dim %d unsupported (32/48/64)", dh); return -1;
  }
}
