// Multi-scale deformable attention v2 sampling core (HBM/L2 gather-bound).
//
// Restates RTDetrV2MultiscaleDeformableAttention.forward M2:166-225 (softmax
// over the L·P attention logits M2:200-203; 4-d reference boxes: loc = ref_xy +
// off · (1/P) · ref_wh · offset_scale, M2:212-215) and the core
// multi_scale_deformable_attention_v2 M2:44-115 (method "default":
// grid_sample(bilinear, zeros, align_corners=False) on 2·loc−1, weighted sum
// over levels × points). The value/offset/weight/output projections run on the
// MFMA GEMM. One workgroup per (image, query); thread (head h, channel c);
// each bilinear corner of a head is one coalesced 32×4 B row segment.
#include "common.h"

namespace sp {
namespace {

__global__ __launch_bounds__(256) void msda_kernel(const sp_msda_desc d) {
  const int t = threadIdx.x;
  const int h = t / d.head_dim;
  const int c = t - h * d.head_dim;
  const int64_t row = blockIdx.x;  // b*Q + q
  const int b = (int)(row / d.Q);
  const int LP = d.levels * d.points;
  const float* offs = d.off_aw + row * d.ld_off_aw + (int64_t)h * LP * 2;
  const float* logit = d.off_aw + row * d.ld_off_aw + (int64_t)d.heads * LP * 2 + (int64_t)h * LP;
  const float rx = d.ref[row * 4 + 0], ry = d.ref[row * 4 + 1];
  const float rw = d.ref[row * 4 + 2], rh = d.ref[row * 4 + 3];
  float mx = -INFINITY;
  for (int i = 0; i < LP; ++i) mx = fmaxf(mx, logit[i]);
  float den = 0.f;
  for (int i = 0; i < LP; ++i) den += expf(logit[i] - mx);
  const float nps = 1.0f / (float)d.points;
  const float* vbase = d.value + (int64_t)b * d.S * d.ld_value + d.value_col + h * d.head_dim + c;
  float out = 0.f;
  for (int l = 0; l < d.levels; ++l) {
    const int H = d.level_h[l], W = d.level_w[l];
    const float* vl = vbase + (int64_t)d.level_start[l] * d.ld_value;
    for (int p = 0; p < d.points; ++p) {
      const int i = l * d.points + p;
      const float a = expf(logit[i] - mx) / den;
      const float lx = rx + offs[2 * i] * nps * rw * d.offset_scale;
      const float ly = ry + offs[2 * i + 1] * nps * rh * d.offset_scale;
      const float gx = 2.0f * lx - 1.0f;
      const float gy = 2.0f * ly - 1.0f;
      const float ix = ((gx + 1.0f) * W - 1.0f) / 2.0f;
      const float iy = ((gy + 1.0f) * H - 1.0f) / 2.0f;
      const float x0 = floorf(ix), y0 = floorf(iy);
      const float x1 = x0 + 1.0f, y1 = y0 + 1.0f;
      const float wnw = (x1 - ix) * (y1 - iy);
      const float wne = (ix - x0) * (y1 - iy);
      const float wsw = (x1 - ix) * (iy - y0);
      const float wse = (ix - x0) * (iy - y0);
      const int xi0 = (int)x0, yi0 = (int)y0;
      const bool vx0 = xi0 >= 0 && xi0 < W, vx1 = xi0 + 1 >= 0 && xi0 + 1 < W;
      const bool vy0 = yi0 >= 0 && yi0 < H, vy1 = yi0 + 1 >= 0 && yi0 + 1 < H;
      float s = 0.f;
      // corner rows of this image's level l: [level_start[l], level_start[l] + H·W) of the B·S value rows
      if (vy0 && vx0) SP_BCHECK((int64_t)b * d.S + d.level_start[l] + (int64_t)yi0 * W + xi0, (int64_t)d.B * d.S);
      if (vy1 && vx1) SP_BCHECK((int64_t)b * d.S + d.level_start[l] + (int64_t)(yi0 + 1) * W + xi0 + 1, (int64_t)d.B * d.S);
      if (vy0 && vx0) s += vl[((int64_t)yi0 * W + xi0) * d.ld_value] * wnw;
      if (vy0 && vx1) s += vl[((int64_t)yi0 * W + xi0 + 1) * d.ld_value] * wne;
      if (vy1 && vx0) s += vl[((int64_t)(yi0 + 1) * W + xi0) * d.ld_value] * wsw;
      if (vy1 && vx1) s += vl[((int64_t)(yi0 + 1) * W + xi0 + 1) * d.ld_value] * wse;
      out += s * a;
    }
  }
  SP_BCHECK(h * d.head_dim + c, d.ld_out);
  d.out[row * d.ld_out + h * d.head_dim + c] = out;
}

// Vectorised form (the decoder's layout: C = heads·Dh with Dh % 4 == 0, 16-byte aligned rows):
// one lane per 4 channels of one head, C/4 lanes per query (64 = one wave per query at C = 256),
// so every bilinear corner is one 16-byte load per lane and a wave-instruction covers the corner
// rows of all 8 heads. Out-of-range corners read a clamped in-range pixel with weight 0 instead of
// branching, so the 4·L·P loads of a lane are independent and stay in flight together. The grid is
// remapped XCD-major: each XCD walks a contiguous run of queries (a few whole images), which keeps
// an image's value rows in that XCD's L2 while its queries are being sampled.
// VBF: the value rows are bf16 (value_bf16, the bf16 variant): each corner is one 8-byte load per lane.
__device__ __forceinline__ float4 corner4(const float* v) { return *reinterpret_cast<const float4*>(v); }
__device__ __forceinline__ float4 corner4(const uint16_t* v) {
  const uint2 u = *reinterpret_cast<const uint2*>(v);
  return make_float4(__builtin_bit_cast(float, u.x << 16), __builtin_bit_cast(float, u.x & 0xffff0000u),
                     __builtin_bit_cast(float, u.y << 16), __builtin_bit_cast(float, u.y & 0xffff0000u));
}

template <typename VT>
__global__ __launch_bounds__(256) void msda_vec_kernel(const sp_msda_desc d, const VT* __restrict__ value,
                                                       int lanes_per_q) {
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int qpw = 256 / lanes_per_q;
  const int64_t row = (int64_t)wg * qpw + threadIdx.x / lanes_per_q;  // b*Q + q
  if (row >= (int64_t)d.B * d.Q) return;
  const int t = threadIdx.x % lanes_per_q;
  const int lph = d.head_dim >> 2;  // lanes per head
  const int h = t / lph;
  const int c = (t - h * lph) * 4;
  const int b = (int)(row / d.Q);
  const int LP = d.levels * d.points;
  const float* offs = d.off_aw + row * d.ld_off_aw + (int64_t)h * LP * 2;
  const float* logit = d.off_aw + row * d.ld_off_aw + (int64_t)d.heads * LP * 2 + (int64_t)h * LP;
  const float rx = d.ref[row * 4 + 0], ry = d.ref[row * 4 + 1];
  const float rw = d.ref[row * 4 + 2], rh = d.ref[row * 4 + 3];
  float mx = -INFINITY;
  for (int i = 0; i < LP; ++i) mx = fmaxf(mx, logit[i]);
  float den = 0.f;
  for (int i = 0; i < LP; ++i) den += expf(logit[i] - mx);
  const float nps = 1.0f / (float)d.points;
  const VT* vbase = value + (int64_t)b * d.S * d.ld_value + d.value_col + h * d.head_dim + c;
  SP_BCHECK(d.value_col + h * d.head_dim + c + 3, d.ld_value);
  SP_BCHECK(h, d.heads);
  float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int l = 0; l < d.levels; ++l) {
    const int H = d.level_h[l], W = d.level_w[l];
    const VT* vl = vbase + (int64_t)d.level_start[l] * d.ld_value;
#pragma unroll 4
    for (int p = 0; p < d.points; ++p) {
      const int i = l * d.points + p;
      const float a = expf(logit[i] - mx) / den;
      const float lx = rx + offs[2 * i] * nps * rw * d.offset_scale;
      const float ly = ry + offs[2 * i + 1] * nps * rh * d.offset_scale;
      const float gx = 2.0f * lx - 1.0f;
      const float gy = 2.0f * ly - 1.0f;
      const float ix = ((gx + 1.0f) * W - 1.0f) / 2.0f;
      const float iy = ((gy + 1.0f) * H - 1.0f) / 2.0f;
      const float x0 = floorf(ix), y0 = floorf(iy);
      const float x1 = x0 + 1.0f, y1 = y0 + 1.0f;
      float wnw = (x1 - ix) * (y1 - iy);
      float wne = (ix - x0) * (y1 - iy);
      float wsw = (x1 - ix) * (iy - y0);
      float wse = (ix - x0) * (iy - y0);
      // far-out locations: keep the integer math in range (every corner is invalid there anyway)
      const int xi0 = (int)fminf(fmaxf(x0, -2.0f), (float)W);
      const int yi0 = (int)fminf(fmaxf(y0, -2.0f), (float)H);
      const bool vx0 = xi0 >= 0 && xi0 < W, vx1 = xi0 + 1 >= 0 && xi0 + 1 < W;
      const bool vy0 = yi0 >= 0 && yi0 < H, vy1 = yi0 + 1 >= 0 && yi0 + 1 < H;
      const int cx0 = min(max(xi0, 0), W - 1), cx1 = min(max(xi0 + 1, 0), W - 1);
      const int cy0 = min(max(yi0, 0), H - 1), cy1 = min(max(yi0 + 1, 0), H - 1);
      // the clamped corners stay inside level l of image b (value rows [b·S, (b+1)·S)), channels inside the row
      SP_BCHECK((int64_t)b * d.S + d.level_start[l] + (int64_t)cy0 * W + cx0, (int64_t)d.B * d.S);
      SP_BCHECK((int64_t)b * d.S + d.level_start[l] + (int64_t)cy1 * W + cx1, (int64_t)d.B * d.S);
      SP_BCHECK(d.level_start[l] + (int64_t)cy1 * W + cx1, d.level_start[l] + (int64_t)H * W);
      const float4 vnw = corner4(vl + ((int64_t)cy0 * W + cx0) * d.ld_value);
      const float4 vne = corner4(vl + ((int64_t)cy0 * W + cx1) * d.ld_value);
      const float4 vsw = corner4(vl + ((int64_t)cy1 * W + cx0) * d.ld_value);
      const float4 vse = corner4(vl + ((int64_t)cy1 * W + cx1) * d.ld_value);
      // an invalid corner adds exactly +0 (same sum as skipping it, M2:79-81 zeros padding)
      wnw = (vy0 && vx0) ? wnw : 0.f;
      wne = (vy0 && vx1) ? wne : 0.f;
      wsw = (vy1 && vx0) ? wsw : 0.f;
      wse = (vy1 && vx1) ? wse : 0.f;
      float4 s;
      s.x = vnw.x * wnw; s.y = vnw.y * wnw; s.z = vnw.z * wnw; s.w = vnw.w * wnw;
      s.x += vne.x * wne; s.y += vne.y * wne; s.z += vne.z * wne; s.w += vne.w * wne;
      s.x += vsw.x * wsw; s.y += vsw.y * wsw; s.z += vsw.z * wsw; s.w += vsw.w * wsw;
      s.x += vse.x * wse; s.y += vse.y * wse; s.z += vse.z * wse; s.w += vse.w * wse;
      out.x += s.x * a; out.y += s.y * a; out.z += s.z * a; out.w += s.w * a;
    }
  }
  SP_BCHECK(h * d.head_dim + c + 3, d.ld_out);
  *reinterpret_cast<float4*>(d.out + row * d.ld_out + h * d.head_dim + c) = out;
}

// The decoder's shape (heads·Dh = 256 → one wave per query, Dh = 32 → 8 lanes per head, L·P = 12): the same
// arithmetic as msda_vec_kernel with the per-point work spread over the 8 lanes of a head instead of repeated by
// each of them. Lane j of a head computes expf of its logits j and j + 8 once (the vec kernel evaluated all 12
// twice per lane) and the location / bilinear weights / clamped corner rows of points j and j + 8, and writes
// them to its wave's LDS slice; every lane of the head then reads each point's record back with two 16-byte and
// one 4-byte LDS reads (the 8 lanes of a head read the same record: an LDS broadcast) and gathers and
// accumulates exactly as the vec kernel does. Same operations in the same order on the same values:
// bit-identical outputs on fp32 value rows (tests/test_gpu_kernels.py::
// test_msda_point_sharing_kernel_is_bit_identical; on bf16 rows the compiler contracts the corner sums into fmas
// differently in the two instantiations: within fp32 rounding). Each wave touches only its own slice, so a
// wave-scope fence orders the writes before the reads (no workgroup barrier; whole waves exit early).
// Round 6 first exchanged the records with cross-lane shuffles (ds_bpermute) instead: bit-identical on a quiet
// GPU, but beside the other micro-batch stream's kernels a few queries per launch came out wrong in one or two
// heads (profiles/r6/msda/insitu_shuffle_exchange.log; root cause not identified). The LDS exchange is exact
// there (tests/test_gpu_model.py::test_two_stream_forward_is_deterministic) and 1.27x faster than the shuffles
// at C2 (profiles/r6/msda/msda_ab.json).
constexpr int kH8Rec = 12;                     // words per point record: rows[4], weights[4], a, pad[3]
constexpr int kH8Head = 12 * kH8Rec + 4;       // words per head (148: the 8 heads' records start 20 banks apart)
constexpr int kH8Wave = 8 * kH8Head + 8 * 16;  // + logits / exponentials, 16 words per head

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename VT>
__global__ __launch_bounds__(256) void msda_h8l_kernel(const sp_msda_desc d, const VT* __restrict__ value) {
  constexpr int LPH = 8, LP = 12, P = 4;
  __shared__ __attribute__((aligned(16))) float sh[4 * kH8Wave];
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int64_t row = (int64_t)wg * 4 + (threadIdx.x >> 6);  // b*Q + q: one query per wave
  if (row >= (int64_t)d.B * d.Q) return;                     // whole waves: no workgroup barrier below
  const int t = threadIdx.x & 63;
  const int h = t >> 3, j = t & 7;
  const int c = j * 4;
  const int b = (int)(row / d.Q);
  float* wsh = sh + (threadIdx.x >> 6) * kH8Wave;
  float* rec = wsh + h * kH8Head;             // this head's 12 point records
  float* lgx = wsh + 8 * kH8Head + h * 16;    // this head's 12 logits, then (reused) exponentials
  const float* offs = d.off_aw + row * d.ld_off_aw + (int64_t)h * LP * 2;
  const float* logit = d.off_aw + row * d.ld_off_aw + (int64_t)d.heads * LP * 2 + (int64_t)h * LP;
  const float rx = d.ref[row * 4 + 0], ry = d.ref[row * 4 + 1];
  const float rw = d.ref[row * 4 + 2], rh = d.ref[row * 4 + 3];
  const int LH0 = d.level_h[0], LH1 = d.level_h[1], LH2 = d.level_h[2];
  const int LW0 = d.level_w[0], LW1 = d.level_w[1], LW2 = d.level_w[2];
  const int LS0 = d.level_start[0], LS1 = d.level_start[1], LS2 = d.level_start[2];
  const bool two = j + LPH < LP;  // lane j owns points j and (for j < 4) j + 8
  const float lg0 = logit[j], lg1 = logit[two ? j + LPH : j];
  lgx[j] = lg0;
  if (two) lgx[j + LPH] = lg1;
  wave_lds_sync();
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < LP; ++i) mx = fmaxf(mx, lgx[i]);
  const float e0 = expf(lg0 - mx), e1 = expf(lg1 - mx);
  wave_lds_sync();  // every lane has read the logits before they are overwritten
  lgx[j] = e0;
  if (two) lgx[j + LPH] = e1;
  wave_lds_sync();
  float den = 0.f;
#pragma unroll
  for (int i = 0; i < LP; ++i) den += lgx[i];  // the vec kernel's order
  const float nps = 1.0f / (float)P;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (k == 1 && !two) break;
    const int ii = j + k * LPH;
    const int l = ii / P;
    const int H = l == 0 ? LH0 : (l == 1 ? LH1 : LH2), W = l == 0 ? LW0 : (l == 1 ? LW1 : LW2);
    const int ls = l == 0 ? LS0 : (l == 1 ? LS1 : LS2);
    const float a = (k == 0 ? e0 : e1) / den;
    const float lx = rx + offs[2 * ii] * nps * rw * d.offset_scale;
    const float ly = ry + offs[2 * ii + 1] * nps * rh * d.offset_scale;
    const float gx = 2.0f * lx - 1.0f;
    const float gy = 2.0f * ly - 1.0f;
    const float ix = ((gx + 1.0f) * W - 1.0f) / 2.0f;
    const float iy = ((gy + 1.0f) * H - 1.0f) / 2.0f;
    const float x0 = floorf(ix), y0 = floorf(iy);
    const float x1 = x0 + 1.0f, y1 = y0 + 1.0f;
    const float wnw = (x1 - ix) * (y1 - iy);
    const float wne = (ix - x0) * (y1 - iy);
    const float wsw = (x1 - ix) * (iy - y0);
    const float wse = (ix - x0) * (iy - y0);
    const int xi0 = (int)fminf(fmaxf(x0, -2.0f), (float)W);
    const int yi0 = (int)fminf(fmaxf(y0, -2.0f), (float)H);
    const bool vx0 = xi0 >= 0 && xi0 < W, vx1 = xi0 + 1 >= 0 && xi0 + 1 < W;
    const bool vy0 = yi0 >= 0 && yi0 < H, vy1 = yi0 + 1 >= 0 && yi0 + 1 < H;
    const int cx0 = min(max(xi0, 0), W - 1), cx1 = min(max(xi0 + 1, 0), W - 1);
    const int cy0 = min(max(yi0, 0), H - 1), cy1 = min(max(yi0 + 1, 0), H - 1);
    SP_BCHECK(ls + cy1 * W + cx1, ls + H * W);
    float* r = rec + ii * kH8Rec;
    *reinterpret_cast<int4*>(r) = make_int4(ls + cy0 * W + cx0, ls + cy0 * W + cx1, ls + cy1 * W + cx0,
                                            ls + cy1 * W + cx1);
    *reinterpret_cast<float4*>(r + 4) = make_float4((vy0 && vx0) ? wnw : 0.f, (vy0 && vx1) ? wne : 0.f,
                                                    (vy1 && vx0) ? wsw : 0.f, (vy1 && vx1) ? wse : 0.f);
    r[8] = a;
  }
  wave_lds_sync();
  const VT* vbase = value + (int64_t)b * d.S * d.ld_value + d.value_col + h * d.head_dim + c;
  SP_BCHECK(d.value_col + h * d.head_dim + c + 3, d.ld_value);
  float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int i = 0; i < LP; ++i) {
    const float* r = rec + i * kH8Rec;
    const int4 rr = *reinterpret_cast<const int4*>(r);
    const float4 w = *reinterpret_cast<const float4*>(r + 4);
    const float a = r[8];
    const float4 vnw = corner4(vbase + (int64_t)rr.x * d.ld_value);
    const float4 vne = corner4(vbase + (int64_t)rr.y * d.ld_value);
    const float4 vsw = corner4(vbase + (int64_t)rr.z * d.ld_value);
    const float4 vse = corner4(vbase + (int64_t)rr.w * d.ld_value);
    float4 s;
    s.x = vnw.x * w.x; s.y = vnw.y * w.x; s.z = vnw.z * w.x; s.w = vnw.w * w.x;
    s.x += vne.x * w.y; s.y += vne.y * w.y; s.z += vne.z * w.y; s.w += vne.w * w.y;
    s.x += vsw.x * w.z; s.y += vsw.y * w.z; s.z += vsw.z * w.z; s.w += vsw.w * w.z;
    s.x += vse.x * w.w; s.y += vse.y * w.w; s.z += vse.z * w.w; s.w += vse.w * w.w;
    out.x += s.x * a; out.y += s.y * a; out.z += s.z * a; out.w += s.w * a;
  }
  SP_BCHECK(h * d.head_dim + c + 3, d.ld_out);
  *reinterpret_cast<float4*>(d.out + row * d.ld_out + h * d.head_dim + c) = out;
}

}  // namespace
}  // namespace sp

namespace sp {
// tuning / test hook: sp_set_tuning(SP_TUNE_MSDA_GENERIC, 1) runs msda_vec_kernel where msda_h8l_kernel applies
static thread_local int g_msda_generic = 0;
int msda_generic() { return g_msda_generic; }
void set_msda_generic(int v) { g_msda_generic = v; }
}  // namespace sp

extern "C" int sp_msda(const sp_msda_desc* d, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(d && (d->value || d->value_bf16) && d->off_aw && d->ref && d->out, "sp_msda: null args");
  SP_ARG_CHECK(d->heads * d->head_dim <= 1024 && (d->heads * d->head_dim) % 64 == 0,
               "sp_msda: heads*head_dim must be a multiple of 64 <= 1024");
  SP_ARG_CHECK(d->levels >= 1 && d->levels <= 4 && d->points >= 1, "sp_msda: levels/points");
  int total = 0;
  for (int l = 0; l < d->levels; ++l) {
    SP_ARG_CHECK(d->level_start[l] == total, "sp_msda: level_start mismatch at %d", l);
    total += d->level_h[l] * d->level_w[l];
  }
  SP_ARG_CHECK(total == d->S, "sp_msda: Σ H·W = %d != S = %d", total, d->S);
  const int C = d->heads * d->head_dim;
  const bool vbf = d->value_bf16 != nullptr;
  const bool vec = d->head_dim % 4 == 0 && 256 % (C / 4) == 0 && d->ld_value % 4 == 0 && d->value_col % 4 == 0 &&
                   d->ld_out % 4 == 0 && ((uintptr_t)(vbf ? (const void*)d->value_bf16 : (const void*)d->value) & (vbf ? 7 : 15)) == 0 &&
                   ((uintptr_t)d->out & 15) == 0;
  SP_ARG_CHECK(vec || !vbf, "sp_msda: bf16 value rows need head_dim %% 4 == 0, aligned rows, C / 4 dividing 256");
  const int64_t rows = (int64_t)d->B * d->Q;
  const bool h8 = vec && C == 256 && d->head_dim == 32 && d->levels == 3 && d->points == 4 && !msda_generic() &&
                  d->ld_off_aw % 4 == 0 && ((uintptr_t)d->off_aw & 15) == 0;
  if (h8) {
    const dim3 grid((unsigned)((rows + 3) / 4));
    if (vbf)
      hipLaunchKernelGGL(msda_h8l_kernel<uint16_t>, grid, dim3(256), 0, as_stream(stream), *d, d->value_bf16);
    else
      hipLaunchKernelGGL(msda_h8l_kernel<float>, grid, dim3(256), 0, as_stream(stream), *d, d->value);
  } else if (vec) {
    const int lanes = C / 4, qpw = 256 / lanes;
    const dim3 grid((unsigned)((rows + qpw - 1) / qpw));
    if (vbf)
      hipLaunchKernelGGL(msda_vec_kernel<uint16_t>, grid, dim3(256), 0, as_stream(stream), *d, d->value_bf16, lanes);
    else
      hipLaunchKernelGGL(msda_vec_kernel<float>, grid, dim3(256), 0, as_stream(stream), *d, d->value, lanes);
  } else {
    hipLaunchKernelGGL(msda_kernel, dim3((unsigned)rows), dim3(C), 0, as_stream(stream), *d);
  }
  return check_launch("sp_msda");
}
