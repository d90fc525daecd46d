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
      if (vy0 && vx0) s += vl[((int64_t)yi0 * W + xi0) * d.ld_value] * wnw;
      if (vy0 && vx1) s += vl[((int64_t)yi0 * W + xi0 + 1) * d.ld_value] * wne;
      if (vy1 && vx0) s += vl[((int64_t)(yi0 + 1) * W + xi0) * d.ld_value] * wsw;
      if (vy1 && vx1) s += vl[((int64_t)(yi0 + 1) * W + xi0 + 1) * d.ld_value] * wse;
      out += s * a;
    }
  }
  d.out[row * d.ld_out + h * d.head_dim + c] = out;
}

}  // namespace
}  // namespace sp

extern "C" int sp_msda(const sp_msda_desc* d, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(d && d->value && d->off_aw && d->ref && d->out, "sp_msda: null args");
  SP_ARG_CHECK(d->heads * d->head_dim <= 1024 && (d->heads * d->head_dim) % 64 == 0,
               "sp_msda: heads*head_dim must be a multiple of 64 <= 1024");
  SP_ARG_CHECK(d->levels >= 1 && d->levels <= 4 && d->points >= 1, "sp_msda: levels/points");
  int total = 0;
  for (int l = 0; l < d->levels; ++l) {
    SP_ARG_CHECK(d->level_start[l] == total, "sp_msda: level_start mismatch at %d", l);
    total += d->level_h[l] * d->level_w[l];
  }
  SP_ARG_CHECK(total == d->S, "sp_msda: Σ H·W = %d != S = %d", total, d->S);
  hipLaunchKernelGGL(msda_kernel, dim3((unsigned)((int64_t)d->B * d->Q)), dim3(d->heads * d->head_dim),
                     0, as_stream(stream), *d);
  return check_launch("sp_msda");
}
