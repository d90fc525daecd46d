// Small fused multi-head self-attention (AIFI: 400 tokens × 8 heads × 48 at 640², 1600 at 1280²;
// decoder: 300 queries × 8 heads × 32): softmax(Q Kᵀ · scale) V. Restates eager_attention_forward /
// sdpa (M2:245-270) as called by RTDetrV2SelfAttention (M2:300-336); the Q/K/V/O projections run on
// the MFMA GEMM (conv_gemm.hip).
//
// Flash-style on the fp32 matrix core (v_mfma_f32_16x16x4_f32: exact fp32 fmaf chains, as the
// GEMMs). One wave owns 16 queries of one (image, head); a 4-wave workgroup shares 64-key K/V tiles
// in LDS. Per 16-key block the wave computes the transposed scores Sᵀ = K Qᵀ (lane l: keys
// 4(l>>4)+i, query l&15), so the online softmax over keys reduces over 4 registers plus two
// cross-group shuffles, and the probabilities are already the B operand of Oᵀ += Vᵀ P: MFMA step s
// pairs lane group g with key 4g+s on both operands (the k order of an MFMA is free), no transpose
// through LDS. Oᵀ lands as 4 consecutive head channels of one query per lane → float4 stores.
#include "common.h"

namespace sp {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int KT = 64;  // keys per LDS tile

// The softmax runs in base 2: the launch folds log2 e into the score scale and the exponentials are v_exp_f32
// (__builtin_amdgcn_exp2f, one instruction instead of expf's range-reduced sequence): the same softmax, within
// 1e-6 of an fp64 reference like the expf form, 1.17-1.28x faster on the C2 / C3 shapes
// (profiles/r4/attn_exp2_ab.jsonl).
// Workgroup → (q-tile, head, image), grouped by XCD: workgroups are dealt round-robin over the 8 XCDs
// (MI355X_MICROARCH.md), so with the q-tile index fastest in the launch order the q-tiles of one (image, head)
// landed on different XCDs and each XCD's L2 fetched that head's K / V on its own. Here XCD x takes the x-th
// contiguous chunk of the work list (q-tile fastest), so the q-tiles of a head share one L2: 1.02-1.04x (fp32)
// and 1.07-1.11x (bf16) at bs32 / bs128, bit-identical (profiles/r5/attn/xcd_*.jsonl). Grids under 512
// workgroups (bs1-bs8) keep the launch order, where grouping measured 1-3 % slower.
__device__ __forceinline__ void attn_work(int n, int heads, int& qtile, int& hh, int& b) {
  const int total = gridDim.x, L = blockIdx.x;
  const int per = total >> 3, rem = total & 7, x = L & 7, i = L >> 3;
  const int w = total < 512 ? L : (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + i;
  const int qt = (n + 63) / 64;
  qtile = w % qt;
  const int r = w / qt;
  hh = r % heads;
  b = r / heads;
}

template <int DH>
__global__ __launch_bounds__(256) void attn_mfma_kernel(const float* __restrict__ q, int64_t ldq,
                                                        const float* __restrict__ k, int64_t ldk,
                                                        const float* __restrict__ v, int64_t ldv,
                                                        float* __restrict__ o, int64_t ldo, int n, int heads,
                                                        float scale) {  // scale: including log2 e
  static_assert(DH % 16 == 0, "head dim in 16-channel blocks");
  constexpr int LD = DH + 4;     // padded LDS row (floats): 16 key rows → distinct bank groups
  constexpr int QS = DH / 4;     // S MFMA steps (k = 4 channels each)
  constexpr int DB = DH / 16;    // 16-channel output blocks
  __shared__ __attribute__((aligned(16))) float Ks[KT * LD];
  __shared__ __attribute__((aligned(16))) float Vs[KT * LD];
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int c16 = lane & 15;
  const int g = lane >> 4;
  int qtile, hh, b;
  attn_work(n, heads, qtile, hh, b);
  const int64_t rowbase = (int64_t)b * n;
  // this head's channels lie inside every operand row (q / k / v may be slices of one fused projection)
  SP_BCHECK(hh * DH + DH - 1, ldq);
  SP_BCHECK(hh * DH + DH - 1, ldk);
  SP_BCHECK(hh * DH + DH - 1, ldv);
  SP_BCHECK(hh * DH + DH - 1, ldo);
  const int q0 = qtile * 64 + wave * 16;
  const int qi = q0 + c16;
  // B operand of Sᵀ = K Qᵀ: step s, lane group g supplies channel g·QS + s of query qi.
  float qv[QS];
  {
    const float* qr = q + (rowbase + (qi < n ? qi : n - 1)) * ldq + hh * DH + g * QS;
#pragma unroll
    for (int c = 0; c < QS; c += 4) {
      const float4 t = *reinterpret_cast<const float4*>(qr + c);
      qv[c] = t.x; qv[c + 1] = t.y; qv[c + 2] = t.z; qv[c + 3] = t.w;
    }
  }
  f32x4 acc[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d) acc[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < n; k0 += KT) {
    const int nk = min(KT, n - k0);
    __syncthreads();
    for (int idx = tid; idx < KT * (DH / 4); idx += 256) {
      const int r = idx / (DH / 4);
      const int c = (idx - r * (DH / 4)) * 4;
      float4 kk = make_float4(0.f, 0.f, 0.f, 0.f), vv = kk;  // rows past nk: zeros (0·p, never NaN)
      if (r < nk) {
        kk = *reinterpret_cast<const float4*>(k + (rowbase + k0 + r) * ldk + hh * DH + c);
        vv = *reinterpret_cast<const float4*>(v + (rowbase + k0 + r) * ldv + hh * DH + c);
      }
      *reinterpret_cast<float4*>(Ks + r * LD + c) = kk;
      *reinterpret_cast<float4*>(Vs + r * LD + c) = vv;
    }
    __syncthreads();
    for (int j0 = 0; j0 < nk; j0 += 16) {
      // Sᵀ block: A = K[key j0 + c16][channel g·QS + s]
      f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f};
      const float* kr = Ks + (j0 + c16) * LD + g * QS;
#pragma unroll
      for (int c = 0; c < QS; c += 4) {
        const float4 t = *reinterpret_cast<const float4*>(kr + c);
        st = __builtin_amdgcn_mfma_f32_16x16x4f32(t.x, qv[c], st, 0, 0, 0);
        st = __builtin_amdgcn_mfma_f32_16x16x4f32(t.y, qv[c + 1], st, 0, 0, 0);
        st = __builtin_amdgcn_mfma_f32_16x16x4f32(t.z, qv[c + 2], st, 0, 0, 0);
        st = __builtin_amdgcn_mfma_f32_16x16x4f32(t.w, qv[c + 3], st, 0, 0, 0);
      }
      // lane holds scores of keys j0 + 4g + i for query qi
      float mt = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        st[i] = (j0 + 4 * g + i < nk) ? st[i] * scale : -INFINITY;
        mt = fmaxf(mt, st[i]);
      }
      mt = fmaxf(mt, __shfl_xor(mt, 16));
      mt = fmaxf(mt, __shfl_xor(mt, 32));
      const float mn = fmaxf(m, mt);
      // first block: m = -inf → 0 (acc, l are 0)
      const float corr = __builtin_amdgcn_exp2f(m - mn);
      m = mn;
      float pr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) pr[i] = __builtin_amdgcn_exp2f(st[i] - mn);
      l = l * corr + ((pr[0] + pr[1]) + (pr[2] + pr[3]));
#pragma unroll
      for (int d = 0; d < DB; ++d) acc[d] *= corr;
      // Oᵀ[channel][query] += Σ_s V[key j0 + 4g + s][channel] · P[key j0 + 4g + s][query]
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float* vr = Vs + (j0 + 4 * g + s) * LD + c16;
#pragma unroll
        for (int d = 0; d < DB; ++d) acc[d] = __builtin_amdgcn_mfma_f32_16x16x4f32(vr[d * 16], pr[s], acc[d], 0, 0, 0);
      }
    }
  }
  // l: this lane group's partial sum over its keys → total over the 4 groups (same query)
  l += __shfl_xor(l, 16);
  l += __shfl_xor(l, 32);
  if (qi >= n) return;
  const float inv = 1.0f / l;
  float* orow = o + (rowbase + qi) * ldo + hh * DH + 4 * g;
#pragma unroll
  for (int d = 0; d < DB; ++d)
    *reinterpret_cast<float4*>(orow + d * 16) =
        make_float4(acc[d][0] * inv, acc[d][1] * inv, acc[d][2] * inv, acc[d][3] * inv);
}

// The bf16 variant's form (round 4): the same flash structure on v_mfma_f32_16x16x16_bf16 — Q, K and V rounded to
// bf16 (RNE) as they are staged, scores and the softmax in fp32, fp32 accumulation. Sᵀ = K Qᵀ takes one MFMA per
// 16 channels (A: key c16, channels 16c + 4g .. +3 from the K tile; B: the lane's query, same channels), so the
// lane again holds keys 4g + i of query c16 and the softmax is the fp32 kernel's. Oᵀ += Vᵀ P takes one MFMA per 16
// output channels: A = V transposed in LDS (channel c16, keys 4g .. 4g + 3: one 8-byte read), B = the lane's four
// probabilities as bf16.
typedef short bf16x4_s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t bf16_pair(float a, float b) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b2));
}

template <int DH>
__global__ __launch_bounds__(256) void attn_bf16_kernel(const float* __restrict__ q, int64_t ldq,
                                                        const float* __restrict__ k, int64_t ldk,
                                                        const float* __restrict__ v, int64_t ldv,
                                                        float* __restrict__ o, int64_t ldo, int n, int heads,
                                                        float scale) {  // scale: including log2 e
  static_assert(DH % 16 == 0, "head dim in 16-channel blocks");
  constexpr int LK = DH + 8;   // K tile row (bf16): 16 rows of a read land on distinct bank pairs
  constexpr int LV = KT + 8;   // Vᵀ tile row (bf16)
  constexpr int QC = DH / 16;  // S MFMAs (16 channels each)
  constexpr int DB = DH / 16;  // 16-channel output blocks
  __shared__ __attribute__((aligned(16))) uint16_t Kb[KT * LK];
  __shared__ __attribute__((aligned(16))) uint16_t Vt[DH * LV];
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int c16 = lane & 15;
  const int g = lane >> 4;
  int qtile, hh, b;
  attn_work(n, heads, qtile, hh, b);
  const int64_t rowbase = (int64_t)b * n;
  // this head's channels lie inside every operand row (q / k / v may be slices of one fused projection)
  SP_BCHECK(hh * DH + DH - 1, ldq);
  SP_BCHECK(hh * DH + DH - 1, ldk);
  SP_BCHECK(hh * DH + DH - 1, ldv);
  SP_BCHECK(hh * DH + DH - 1, ldo);
  const int qi = qtile * 64 + wave * 16 + c16;
  bf16x4_s qv[QC];  // channels 16c + 4g .. +3 of query qi
  {
    const float* qr = q + (rowbase + (qi < n ? qi : n - 1)) * ldq + hh * DH + 4 * g;
#pragma unroll
    for (int c = 0; c < QC; ++c) {
      const float4 t = *reinterpret_cast<const float4*>(qr + 16 * c);
      const uint2 u = make_uint2(bf16_pair(t.x, t.y), bf16_pair(t.z, t.w));
      qv[c] = __builtin_bit_cast(bf16x4_s, u);
    }
  }
  f32x4 acc[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d) acc[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < n; k0 += KT) {
    const int nk = min(KT, n - k0);
    __syncthreads();
    for (int idx = tid; idx < KT * (DH / 4); idx += 256) {
      const int r = idx / (DH / 4);
      const int c = (idx - r * (DH / 4)) * 4;
      float4 kk = make_float4(0.f, 0.f, 0.f, 0.f), vv = kk;  // rows past nk: zeros (0·p, never NaN)
      if (r < nk) {
        kk = *reinterpret_cast<const float4*>(k + (rowbase + k0 + r) * ldk + hh * DH + c);
        vv = *reinterpret_cast<const float4*>(v + (rowbase + k0 + r) * ldv + hh * DH + c);
      }
      *reinterpret_cast<uint2*>(Kb + r * LK + c) = make_uint2(bf16_pair(kk.x, kk.y), bf16_pair(kk.z, kk.w));
      const uint32_t v01 = bf16_pair(vv.x, vv.y), v23 = bf16_pair(vv.z, vv.w);
      Vt[(c + 0) * LV + r] = (uint16_t)(v01 & 0xffffu);
      Vt[(c + 1) * LV + r] = (uint16_t)(v01 >> 16);
      Vt[(c + 2) * LV + r] = (uint16_t)(v23 & 0xffffu);
      Vt[(c + 3) * LV + r] = (uint16_t)(v23 >> 16);
    }
    __syncthreads();
    for (int j0 = 0; j0 < nk; j0 += 16) {
      f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < QC; ++c) {
        const bf16x4_s a = *reinterpret_cast<const bf16x4_s*>(Kb + (j0 + c16) * LK + 16 * c + 4 * g);
        st = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, qv[c], st, 0, 0, 0);
      }
      float mt = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        st[i] = (j0 + 4 * g + i < nk) ? st[i] * scale : -INFINITY;
        mt = fmaxf(mt, st[i]);
      }
      mt = fmaxf(mt, __shfl_xor(mt, 16));
      mt = fmaxf(mt, __shfl_xor(mt, 32));
      const float mn = fmaxf(m, mt);
      const float corr = __builtin_amdgcn_exp2f(m - mn);
      m = mn;
      float pr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) pr[i] = __builtin_amdgcn_exp2f(st[i] - mn);
      l = l * corr + ((pr[0] + pr[1]) + (pr[2] + pr[3]));
#pragma unroll
      for (int d = 0; d < DB; ++d) acc[d] *= corr;
      const bf16x4_s pb = __builtin_bit_cast(bf16x4_s, make_uint2(bf16_pair(pr[0], pr[1]), bf16_pair(pr[2], pr[3])));
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        const bf16x4_s a = *reinterpret_cast<const bf16x4_s*>(Vt + (16 * d + c16) * LV + j0 + 4 * g);
        acc[d] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, pb, acc[d], 0, 0, 0);
      }
    }
  }
  l += __shfl_xor(l, 16);
  l += __shfl_xor(l, 32);
  if (qi >= n) return;
  const float inv = 1.0f / l;
  float* orow = o + (rowbase + qi) * ldo + hh * DH + 4 * g;
#pragma unroll
  for (int d = 0; d < DB; ++d)
    *reinterpret_cast<float4*>(orow + d * 16) =
        make_float4(acc[d][0] * inv, acc[d][1] * inv, acc[d][2] * inv, acc[d][3] * inv);
}

template <int DH, bool BF>
int launch(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v, int64_t ldv,
           float* o, int64_t ldo, int batch, int n, int heads, float scale, hipStream_t s) {
  const int64_t wgs = (int64_t)((n + 63) / 64) * heads * batch;  // one workgroup per 64 queries of a head
  if (wgs > 0x7fffffff) {
    set_error("sp_attention: %lld workgroups", (long long)wgs);
    return -1;
  }
  dim3 grid((unsigned)wgs);
  if constexpr (BF)
    hipLaunchKernelGGL((attn_bf16_kernel<DH>), grid, dim3(256), 0, s, q, ldq, k, ldk, v, ldv, o, ldo, n, heads,
                       scale * 1.4426950408889634f);  // log2 e: the softmax in base 2
  else
    hipLaunchKernelGGL((attn_mfma_kernel<DH>), grid, dim3(256), 0, s, q, ldq, k, ldk, v, ldv, o, ldo, n, heads,
                       scale * 1.4426950408889634f);
  return check_launch(BF ? "sp_attention_bf16" : "sp_attention");
}

template <bool BF>
int attention(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v, int64_t ldv, float* o,
              int64_t ldo, int batch, int n, int heads, int dh, float scale, void* stream) {
  SP_ARG_CHECK(q && k && v && o && batch > 0 && n > 0 && heads > 0, "sp_attention: bad args");
  SP_ARG_CHECK(ldq % 4 == 0 && ldk % 4 == 0 && ldv % 4 == 0 && ldo % 4 == 0, "sp_attention: ld % 4");
  hipStream_t s = as_stream(stream);
  switch (dh) {
    case 32: return launch<32, BF>(q, ldq, k, ldk, v, ldv, o, ldo, batch, n, heads, scale, s);
    case 48: return launch<48, BF>(q, ldq, k, ldk, v, ldv, o, ldo, batch, n, heads, scale, s);
    case 64: return launch<64, BF>(q, ldq, k, ldk, v, ldv, o, ldo, batch, n, heads, scale, s);
    default: set_error("sp_attention: head_dim %d unsupported (32/48/64)", dh); return -1;
  }
}

}  // namespace
}  // namespace sp

extern "C" int sp_attention(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v,
                            int64_t ldv, float* o, int64_t ldo, int batch, int n, int heads, int dh,
                            float scale, void* stream) {
  return sp::attention<false>(q, ldq, k, ldk, v, ldv, o, ldo, batch, n, heads, dh, scale, stream);
}

extern "C" int sp_attention_bf16(const float* q, int64_t ldq, const float* k, int64_t ldk, const float* v,
                                 int64_t ldv, float* o, int64_t ldo, int batch, int n, int heads, int dh,
                                 float scale, void* stream) {
  return sp::attention<true>(q, ldq, k, ldk, v, ldv, o, ldo, batch, n, heads, dh, scale, stream);
}
