// Per-row top-k by radix select (query selection and post-process).
//
// Query selection: torch.topk(enc_outputs_class.max(-1).values, 300) over the
// 8,400 anchors at 640² (M2:1599). Post-process: torch.topk(sigmoid(logits)
// .flatten(1), 300) over 300×80 (IPP:555-556), then label = i % C, query =
// i // C, cxcywh→xyxy (IT:529-536) scaled by the original (w, h, w, h)
// (IPP:538-549), keep score > threshold (IPP:572-574).
//
// One 1024-thread workgroup per row: keys (order-preserving uint32 of the
// fp32 value, after the optional max-over-C reduction / sigmoid) live in LDS
// (≤ 36,864 per row); four 8-bit radix passes find the k-th largest key T;
// keys > T are compacted, keys == T are taken in index order; each winner's rank
// under (key desc, index asc) places it. Deterministic.
#include "common.h"

namespace sp {
namespace {

constexpr int kThreads = 1024;
constexpr int kMaxN = 36864;  // 144 KiB of keys: covers S = 33,600 at 1280² (LDS 160 KiB)
constexpr int kMaxK = 512;
constexpr int kHist = 4;  // histogram copies (LDS: keys 144 KiB + 4 KiB + candidates 4 KiB)

__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

__global__ __launch_bounds__(kThreads) void topk_kernel(const float* __restrict__ x, int64_t ldx, int n,
                                                         int reduce_c, int apply_sigmoid, int k,
                                                         float* __restrict__ vals,
                                                         int32_t* __restrict__ idx_out) {
  __shared__ uint32_t keys[kMaxN];
  __shared__ uint32_t hist[kHist][256];  // privatised per wave group: sigmoid/logit keys share few top bytes
  __shared__ unsigned long long cand[kMaxK];
  __shared__ uint32_t s_sel[4];  // prefix, remaining, count_gt, count_eq
  __shared__ uint32_t wave_tot[kThreads / 64];

  const int tid = threadIdx.x;
  const int64_t row = blockIdx.x;
  const float* xr = x + row * ldx;
  const int G4 = reduce_c / 4;
  const bool coalesced = reduce_c > 1 && reduce_c % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0;
  if (coalesced) {
    // max over each group of reduce_c classes: a wave covers 16 groups per step, lane (part p = l >> 4,
    // group g = l & 15) loading float4s p, p+4, p+8, ... of group g — every wave-instruction reads
    // 16 × 64 contiguous bytes — then two xor-shuffles fold the 4 parts (max is order-independent).
    // Two steps are in flight per iteration.
    const int w = tid >> 6, ln = tid & 63, g = ln & 15, part = ln >> 4;
    const float4* xr4 = reinterpret_cast<const float4*>(xr);
    constexpr int kW = kThreads / 64;
    for (int g0 = w * 32; g0 < n; g0 += kW * 32) {
      float m2[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int grp = g0 + 16 * u + g;
        float m = -INFINITY;
        if (grp < n) {
          const float4* q = xr4 + (int64_t)grp * G4;
          for (int t = part; t < G4; t += 4) {
            const float4 v = q[t];
            m = fmaxf(m, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
          }
        }
        m2[u] = m;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float m = m2[u];
        m = fmaxf(m, __shfl_xor(m, 16));
        m = fmaxf(m, __shfl_xor(m, 32));
        const int grp = g0 + 16 * u + g;
        if (part == 0 && grp < n) {
          if (apply_sigmoid) m = sigmoidf_(m);
          keys[grp] = f2key(m);
        }
      }
    }
  }
  for (int i = tid; i < n && !coalesced; i += kThreads) {
    float v;
    if (reduce_c > 1) {
      const float* p = xr + (int64_t)i * reduce_c;
      v = p[0];
      for (int c = 1; c < reduce_c; ++c) v = fmaxf(v, p[c]);
    } else {
      v = xr[i];
    }
    if (apply_sigmoid) v = sigmoidf_(v);
    keys[i] = f2key(v);
  }
  for (int i = tid; i < kMaxK; i += kThreads) cand[i] = 0ull;
  if (tid == 0) { s_sel[0] = 0; s_sel[1] = (uint32_t)k; s_sel[2] = 0; s_sel[3] = 0; }
  __syncthreads();

  uint32_t mask = 0;
  uint32_t* my_hist = hist[(tid >> 6) % kHist];
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = tid; i < kHist * 256; i += kThreads) (&hist[0][0])[i] = 0;
    __syncthreads();
    const uint32_t prefix = s_sel[0];
    const uint32_t rem = s_sel[1];  // read before the selecting thread rewrites it below
    // keys that survived the earlier digits crowd into a few bins (sigmoid scores share their top bytes),
    // so each wave adds its most common case — the lanes matching the first live lane's digit — with one
    // atomic, and only the other lanes add their own
    for (int i = tid; i < n; i += kThreads) {
      const uint32_t key = keys[i];
      const bool live = (key & mask) == prefix;
      const uint32_t dg = (key >> shift) & 255u;
      const unsigned long long act = __ballot(live);
      if (act) {
        const int lead = __ffsll((long long)act) - 1;
        const uint32_t ld = __shfl(dg, lead);
        const bool same = live && dg == ld;
        const unsigned long long sm = __ballot(same);
        if (live && !same) atomicAdd(&my_hist[dg], 1u);
        if ((tid & 63) == lead) atomicAdd(&my_hist[ld], (uint32_t)__popcll(sm));
      }
    }
    __syncthreads();
    // the digit of the k-th largest key: bin b with above(b) < rem <= above(b) + hist(b), where above(b)
    // = Σ hist over bins > b — a suffix scan over the 256 bins in four waves (shuffles + 4 wave totals)
    // instead of one thread walking the bins
    uint32_t tot = 0, suf = 0;
    if (tid < 256) {
      for (int j = 0; j < kHist; ++j) tot += hist[j][tid];
      suf = tot;  // becomes Σ hist over bins >= tid within this wave
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_down(suf, off);
        if ((tid & 63) + off < 64) suf += t;
      }
      if ((tid & 63) == 0) wave_tot[tid >> 6] = suf;
    }
    __syncthreads();
    if (tid < 256) {
      for (int w = (tid >> 6) + 1; w < 4; ++w) suf += wave_tot[w];
      const uint32_t above = suf - tot;
      if (above < rem && rem <= suf) {
        s_sel[0] = prefix | ((uint32_t)tid << shift);
        s_sel[1] = rem - above;
      }
    }
    mask |= 255u << shift;
    __syncthreads();
  }
  const uint32_t T = s_sel[0];
  const uint32_t need_eq = s_sel[1];
  const uint32_t n_gt = (uint32_t)k - need_eq;
  // keys > T: any order (ranked below); count the keys == T alongside
  for (int i = tid; i < n; i += kThreads) {
    const uint32_t key = keys[i];
    if (key > T) {
      const uint32_t pos = atomicAdd(&s_sel[2], 1u);
      SP_BCHECK(pos, k);  // exactly n_gt = k - need_eq keys lie above the threshold key
      cand[pos] = ((unsigned long long)key << 32) | (0xffffffffu - (uint32_t)i);
    } else if (key == T) {
      atomicAdd(&s_sel[3], 1u);
    }
  }
  __syncthreads();
  if (s_sel[3] == need_eq) {
    // every key == T is taken (no tie across the cut): append them in any order after the n_gt above
    for (int i = tid; i < n; i += kThreads)
      if (keys[i] == T) {
        const uint32_t pos = atomicAdd(&s_sel[2], 1u);
        SP_BCHECK(pos, k);
        cand[pos] = ((unsigned long long)T << 32) | (0xffffffffu - (uint32_t)i);
      }
  } else {
    // a tie across the cut: the first need_eq keys == T in index order (ordered block compaction)
    const int lane = tid & 63, wid = tid >> 6;
    uint32_t taken = 0;
    for (int base = 0; base < n && taken < need_eq; base += kThreads) {
      const int i = base + tid;
      const bool f = i < n && keys[i] == T;
      const unsigned long long bal = __ballot(f);
      const uint32_t before = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
      if (lane == 0) wave_tot[wid] = (uint32_t)__popcll(bal);
      __syncthreads();
      uint32_t off = 0, tot = 0;
      for (int w = 0; w < kThreads / 64; ++w) {
        if (w < wid) off += wave_tot[w];
        tot += wave_tot[w];
      }
      const uint32_t pos = taken + off + before;
      if (f && pos < need_eq)
        cand[n_gt + pos] = ((unsigned long long)T << 32) | (0xffffffffu - (uint32_t)i);
      taken += tot;
      __syncthreads();
    }
  }
  __syncthreads();
  // order the k winners by (key desc, index asc): every entry is distinct (the index is in the low word),
  // so its position is the number of entries greater than it — one pass of broadcast LDS reads per
  // thread, no sorting network
  for (int i = tid; i < k; i += kThreads) {
    const unsigned long long e = cand[i];
    int rank = 0;
    for (int j = 0; j < k; ++j) rank += cand[j] > e;
    const uint32_t key = (uint32_t)(e >> 32);
    const uint32_t id = 0xffffffffu - (uint32_t)(e & 0xffffffffu);
    SP_BCHECK(rank, k);
    SP_BCHECK(id, n);  // an unfilled candidate slot (0) would decode to index 2^32 - 1
    idx_out[row * k + rank] = (int32_t)id;
    if (vals) vals[row * k + rank] = key2f(key);
  }
}

__global__ __launch_bounds__(512) void decode_kernel(const float* __restrict__ boxes, const int32_t* __restrict__ target_hw,
                                                     int q, int c, int k, float thr,
                                                     const float* __restrict__ scores, const int32_t* __restrict__ idx,
                                                     int64_t* __restrict__ labels, float* __restrict__ out_boxes,
                                                     int32_t* __restrict__ counts) {
  __shared__ int s_cnt;
  const int b = blockIdx.x;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  const float ih = (float)target_hw[2 * b], iw = (float)target_hw[2 * b + 1];
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    const int32_t id = idx[(int64_t)b * k + i];
    SP_BCHECK(id, (int64_t)q * c);
    const int lab = id % c;
    const int qq = id / c;
    const float* bx = boxes + ((int64_t)b * q + qq) * 4;
    const float cx = bx[0], cy = bx[1], w = bx[2], h = bx[3];
    float* o = out_boxes + ((int64_t)b * k + i) * 4;
    o[0] = (cx - 0.5f * w) * iw;
    o[1] = (cy - 0.5f * h) * ih;
    o[2] = (cx + 0.5f * w) * iw;
    o[3] = (cy + 0.5f * h) * ih;
    labels[(int64_t)b * k + i] = lab;
    if (scores[(int64_t)b * k + i] > thr) atomicAdd(&s_cnt, 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) counts[b] = s_cnt;
}

// Per-anchor max over the class logits (the reduction in front of query selection's top-k, M2:1599),
// spread over the whole chip: 4 lanes per row, float4 loads, two xor-shuffles. The top-k kernel then
// works on one key per anchor instead of streaming the [S, C] logits through a single workgroup.
__global__ __launch_bounds__(256) void rowmax4_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows,
                                                      int c4, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r = t >> 2;
  const int part = (int)(t & 3);
  float m = -INFINITY;
  if (r < rows) {
    const float4* q = reinterpret_cast<const float4*>(x + r * ldx);
    for (int j = part; j < c4; j += 4) {
      const float4 v = q[j];
      m = fmaxf(m, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    }
  }
  m = fmaxf(m, __shfl_xor(m, 1));
  m = fmaxf(m, __shfl_xor(m, 2));
  if (r < rows && part == 0) out[r] = m;
}

__global__ __launch_bounds__(256) void rowmax_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows, int c,
                                                     float* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= rows) return;
  const float* q = x + r * ldx;
  float m = q[0];
  for (int j = 1; j < c; ++j) m = fmaxf(m, q[j]);
  out[r] = m;
}

}  // namespace
}  // namespace sp

extern "C" int sp_rowmax(const float* x, int64_t ldx, int64_t rows, int c, float* out, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(x && out && rows > 0 && c > 0 && ldx >= c, "sp_rowmax: bad args");
  hipStream_t s = as_stream(stream);
  if (c % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0) {
    const int64_t g = (rows * 4 + 255) / 256;
    SP_ARG_CHECK(g <= 0x7fffffff, "sp_rowmax: rows");
    hipLaunchKernelGGL(rowmax4_kernel, dim3((unsigned)g), dim3(256), 0, s, x, ldx, rows, c / 4, out);
  } else {
    const int64_t g = (rows + 255) / 256;
    SP_ARG_CHECK(g <= 0x7fffffff, "sp_rowmax: rows");
    hipLaunchKernelGGL(rowmax_kernel, dim3((unsigned)g), dim3(256), 0, s, x, ldx, rows, c, out);
  }
  return check_launch("sp_rowmax");
}

extern "C" int sp_topk_rows(const float* x, int64_t ldx, int rows, int n, int reduce_c, int apply_sigmoid,
                            int k, float* vals, int32_t* idx, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(x && idx && rows > 0 && n > 0, "sp_topk_rows: bad args");
  SP_ARG_CHECK(n <= kMaxN, "sp_topk_rows: n=%d > %d", n, kMaxN);
  SP_ARG_CHECK(k > 0 && k <= kMaxK && k <= n, "sp_topk_rows: k=%d (n=%d, max %d)", k, n, kMaxK);
  SP_ARG_CHECK(reduce_c >= 1, "sp_topk_rows: reduce_c");
  hipLaunchKernelGGL(topk_kernel, dim3(rows), dim3(kThreads), 0, as_stream(stream), x, ldx, n, reduce_c,
                     apply_sigmoid, k, vals, idx);
  return check_launch("sp_topk_rows");
}

extern "C" int sp_postprocess(const float* logits, const float* boxes, const int32_t* target_hw, int batch,
                              int q, int c, int k, float threshold, float* scores, int64_t* labels,
                              float* boxes_xyxy, int32_t* counts, int32_t* work, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(logits && boxes && target_hw && scores && labels && boxes_xyxy && counts && work,
               "sp_postprocess: null args");
  int rc = sp_topk_rows(logits, (int64_t)q * c, batch, q * c, 1, 1, k, scores, work, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(decode_kernel, dim3(batch), dim3(512), 0, as_stream(stream), boxes, target_hw, q, c, k,
                     threshold, scores, work, labels, boxes_xyxy, counts);
  return check_launch("sp_postprocess");
}
