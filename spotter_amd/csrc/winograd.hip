// 3×3 stride-1 convolution by Winograd F(2×2, 3×3) on the fp32-accurate split GEMM.
//
// A 3×3 conv (M2:817-835 ConvNormLayer / M2:921-923 the re-parameterised RepVGG conv, RN:78-103 the
// ResNet 3×3s) computes out = act(Σ_taps x·w · scale + shift + res1) + res2. With 2×2 output tiles
// (4×4 input patches d, rows/cols 2t-1 .. 2t+2, zero padding) it factors into
//   V = Bᵀ d B              (input transform, sp per tile and channel, only ± additions),
//   M_ab = Σ_ci V_ab · U_ab   (16 independent GEMMs [tiles × Cin] · [Cin × Cout], U = G g Gᵀ on the host),
//   Y = Aᵀ M A               (output transform, ± additions) → the usual epilogue.
// The GEMMs carry 16/36 of the direct conv's multiply-adds (2.25× fewer) and run on the batched
// LDS-DMA kernels of conv_glds.hip in any operand mode (x3 split: fp32-accurate; bf16). In fp32 the
// transforms add two roundings on each side; the error measured against fp64 matches the direct fp32
// conv's (the GEMM's K is 9× shorter) — tests/test_gpu_kernels.py::test_winograd_*.
//
// Layout: V [16][T][Cin] and M [16][T][Cout] fp32 in the caller's workspace, T = N·⌈H/2⌉·⌈W/2⌉ tiles
// (b, ty, tx) row-major; component ab = 4a + b. The transform kernels are HBM-bound streams with
// consecutive threads on consecutive 4-channel groups: the input transform takes two adjacent tiles
// per thread (24 float4 loads, 32 float4 stores), the output transform one tile (16 non-temporal
// float4 loads, 4 float4 stores + the epilogue's residual loads).
#include <cstdlib>
#include "mfma16_common.h"

namespace sp {
namespace {

typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 ld_nt(const float* p) {
  const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}

// Input transform, two horizontally adjacent tiles per thread: their 4×4 patches share two columns,
// so 24 loads (4 rows × 6 columns) feed 2 × 16 outputs (profiles/r2/wino_transforms_ab.json: on par
// with one tile per thread, a little ahead at 80² and 20²; non-temporal V stores measured slower).
__global__ __launch_bounds__(256) void wino_in_f23_x2_kernel(const float* __restrict__ x, int64_t lda, int h, int w,
                                                             int c4n, int th, int tw, int64_t nb,
                                                             float* __restrict__ V, int64_t cin) {
  const int tw2 = (tw + 1) / 2;
  const int64_t T = nb * th * tw;
  const int64_t total = nb * th * tw2 * c4n;
  const int64_t plane = T * cin;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t2 = g / c4n;
    const int c = (int)(g - t2 * c4n) * 4;
    const int64_t b = t2 / ((int64_t)th * tw2);
    const int r = (int)(t2 - b * th * tw2);
    const int ty = r / tw2;
    const int tx0 = 2 * (r - ty * tw2);
    const int y0 = 2 * ty - 1, x0 = 2 * tx0 - 1;
    float4 d[4][6];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int yy = y0 + i, xx = x0 + j;
        if ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w) SP_BCHECK((b * h + yy) * w + xx, nb * h * w);
        d[i][j] = ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w)
                      ? *reinterpret_cast<const float4*>(x + ((b * h + yy) * w + xx) * lda + c)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (tx0 + k >= tw) break;
      float4 q[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        q[i][0] = d[i][2 * k + 0] - d[i][2 * k + 2];
        q[i][1] = d[i][2 * k + 1] + d[i][2 * k + 2];
        q[i][2] = d[i][2 * k + 2] - d[i][2 * k + 1];
        q[i][3] = d[i][2 * k + 1] - d[i][2 * k + 3];
      }
      SP_BCHECK((b * th + ty) * tw + tx0 + k, T);
      SP_BCHECK(c + 3, cin);
      float* dst = V + ((b * th + ty) * tw + tx0 + k) * cin + c;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        *reinterpret_cast<float4*>(dst + (0 * 4 + bb) * plane) = q[0][bb] - q[2][bb];
        *reinterpret_cast<float4*>(dst + (1 * 4 + bb) * plane) = q[1][bb] + q[2][bb];
        *reinterpret_cast<float4*>(dst + (2 * 4 + bb) * plane) = q[2][bb] - q[1][bb];
        *reinterpret_cast<float4*>(dst + (3 * 4 + bb) * plane) = q[1][bb] - q[3][bb];
      }
    }
  }
}

__device__ __forceinline__ float4 epi4(float4 v, const sp_conv_desc& d, int64_t m, int n) {
  const float4 sc = d.scale ? *reinterpret_cast<const float4*>(d.scale + n) : make_float4(1.f, 1.f, 1.f, 1.f);
  const float4 sh = d.shift ? *reinterpret_cast<const float4*>(d.shift + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  v.x = fmaf(v.x, sc.x, sh.x); v.y = fmaf(v.y, sc.y, sh.y);
  v.z = fmaf(v.z, sc.z, sh.z); v.w = fmaf(v.w, sc.w, sh.w);
  if (d.res1) {
    const float4 a = *reinterpret_cast<const float4*>(d.res1 + m * d.ldr1 + n);
    v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
  }
  v.x = act_apply(v.x, d.act); v.y = act_apply(v.y, d.act);
  v.z = act_apply(v.z, d.act); v.w = act_apply(v.w, d.act);
  if (d.res2) {
    const float4 a = *reinterpret_cast<const float4*>(d.res2 + m * d.ldr2 + n);
    v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
  }
  return v;
}

__global__ __launch_bounds__(256) void wino_out_f23_kernel(const float* __restrict__ Mc, int64_t T, int c4n,
                                                           int th, int tw, const sp_conv_desc d) {
  const int64_t total = T * c4n;
  const int64_t cout = d.Cout;
  const int64_t plane = T * cout;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = g / c4n;
    const int n = (int)(g - t * c4n) * 4;
    const int64_t b = t / ((int64_t)th * tw);
    const int r = (int)(t - b * th * tw);
    const int ty = r / tw;
    const int tx = r - ty * tw;
    SP_BCHECK(n + 3, cout);
    const float* src = Mc + t * cout + n;
    float4 mm[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) mm[a][bb] = ld_nt(src + (a * 4 + bb) * plane);  // read once: +15-20 %
    // Aᵀ = [[1,1,1,0],[0,1,-1,-1]]: s = Aᵀ M (over a), then Y = s A (over b)
    float4 s[2][4];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      s[0][bb] = mm[0][bb] + mm[1][bb] + mm[2][bb];
      s[1][bb] = mm[1][bb] - mm[2][bb] - mm[3][bb];
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int oy = 2 * ty + p;
      if (oy >= d.Ho) break;
      const float4 y0 = s[p][0] + s[p][1] + s[p][2];
      const float4 y1 = s[p][1] - s[p][2] - s[p][3];
      const int64_t m0 = (b * d.Ho + oy) * d.Wo + 2 * tx;
      SP_BCHECK(m0, (int64_t)d.N * d.Ho * d.Wo);
      *reinterpret_cast<float4*>(d.C + m0 * d.ldc + n) = epi4(y0, d, m0, n);
      if (2 * tx + 1 < d.Wo) *reinterpret_cast<float4*>(d.C + (m0 + 1) * d.ldc + n) = epi4(y1, d, m0 + 1, n);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// F(4×4, 3×3) on the interpolation points (0, -1, 1, ½, -2, ∞): 6×6 input patches (rows / cols
// 4t-1 .. 4t+4), 36 components, 36/(16·9) = 1/4 of the direct conv's multiply-adds. The points are
// chosen for fp32 error (numpy study, DESIGN §4: max |e| / Σ|ab| 3.6e-7 vs 1.0e-6 for the common
// (0, ±1, ±2) set and 7.7e-8 for the direct conv); Bᵀ and Aᵀ hold small dyadic values (exact in fp32),
// G (thirds, fifteenths) is applied in fp64 on the host.
constexpr float kBT43[6][6] = {{1.f, -1.5f, -2.f, 1.5f, 1.f, 0.f},  {0.f, 1.f, -2.5f, 0.5f, 1.f, 0.f},
                               {0.f, -1.f, 0.5f, 2.5f, 1.f, 0.f},   {0.f, -2.f, -1.f, 2.f, 1.f, 0.f},
                               {0.f, 0.5f, -1.f, -0.5f, 1.f, 0.f},  {0.f, 1.f, -1.5f, -2.f, 1.5f, 1.f}};
constexpr float kAT43[4][6] = {{1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
                               {0.f, -1.f, 1.f, 0.5f, -2.f, 0.f},
                               {0.f, 1.f, 1.f, 0.25f, 4.f, 0.f},
                               {0.f, -1.f, 1.f, 0.125f, -8.f, 1.f}};

template <int VW>
struct VT {
  typedef float type __attribute__((ext_vector_type(VW)));
};

// VW consecutive channels per thread (1 or 2: the launch takes 1 on maps too small to fill the chip
// with 2-channel threads).
// V element (component k, tile t, channel c) lives at V[k·cstride + t·tstride + c]: component-major,
// cstride = T·Cin, tstride = Cin. (Round 4 measured the tile-major layout — the 36 components of a tile
// side by side — non-temporal map loads / V stores, and 2-8 tile rows per thread sharing the patch
// overlap: within ±1 % or slower on the C2 shapes, profiles/r4/wino/.)
template <int VW>
__global__ __launch_bounds__(256) void wino_in_f43_kernel(const float* __restrict__ x, int64_t lda, int h, int w,
                                                          int cvn, int th, int tw, int64_t T,
                                                          float* __restrict__ V, int64_t tstride, int64_t cstride) {
  typedef typename VT<VW>::type vf;
  const int64_t total = T * cvn;
  const int64_t plane = cstride;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = g / cvn;
    const int c = (int)(g - t * cvn) * VW;
    const int64_t b = t / ((int64_t)th * tw);
    const int r = (int)(t - b * th * tw);
    const int ty = r / tw;
    const int tx = r - ty * tw;
    const int y0 = 4 * ty - 1, x0 = 4 * tx - 1;
    vf q[6][6];  // row pass: q[i][bb] = Σ_j Bᵀ[bb][j] d[i][j]
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      vf dr[6];
      const int yy = y0 + i;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int xx = x0 + j;
        if ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w) SP_BCHECK((b * h + yy) * w + xx, (T / ((int64_t)th * tw)) * h * w);
        dr[j] = ((unsigned)yy < (unsigned)h && (unsigned)xx < (unsigned)w)
                    ? *reinterpret_cast<const vf*>(x + ((b * h + yy) * w + xx) * lda + c)
                    : vf(0.f);
      }
#pragma unroll
      for (int bb = 0; bb < 6; ++bb) {
        vf acc = vf(0.f);
#pragma unroll
        for (int j = 0; j < 6; ++j)
          if (kBT43[bb][j] != 0.f) acc = __builtin_elementwise_fma(vf(kBT43[bb][j]), dr[j], acc);
        q[i][bb] = acc;
      }
    }
    float* dst = V + t * tstride + c;
    // the last component's element of this (tile, channel group) inside the 36·T·Cin V region
    SP_BCHECK(35 * plane + t * tstride + c + VW - 1, 36 * plane);
    SP_BCHECK(c + VW - 1, tstride);
#pragma unroll
    for (int bb = 0; bb < 6; ++bb)
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        vf v = vf(0.f);
#pragma unroll
        for (int i = 0; i < 6; ++i)
          if (kBT43[a][i] != 0.f) v = __builtin_elementwise_fma(vf(kBT43[a][i]), q[i][bb], v);
        *reinterpret_cast<vf*>(dst + (a * 6 + bb) * plane) = v;
      }
  }
}

template <int VW>
__global__ __launch_bounds__(256) void wino_out_f43_kernel(const float* __restrict__ Mc, int64_t T, int cvn,
                                                           int th, int tw, const sp_conv_desc d, int64_t tstride,
                                                           int64_t cstride) {
  typedef typename VT<VW>::type vf;
  const int64_t total = T * cvn;
  const int64_t plane = cstride;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < total; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = g / cvn;
    const int n = (int)(g - t * cvn) * VW;
    const int64_t b = t / ((int64_t)th * tw);
    const int r = (int)(t - b * th * tw);
    const int ty = r / tw;
    const int tx = r - ty * tw;
    const float* src = Mc + t * tstride + n;
    SP_BCHECK(35 * plane + t * tstride + n + VW - 1, 36 * plane);
    SP_BCHECK(n + VW - 1, d.Cout);
    vf s[4][6];  // s[p][bb] = Σ_a Aᵀ[p][a] M[a][bb], accumulated as the rows of M arrive
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int bb = 0; bb < 6; ++bb) s[p][bb] = vf(0.f);
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      vf mr[6];
#pragma unroll
      for (int bb = 0; bb < 6; ++bb)
        mr[bb] = __builtin_nontemporal_load(reinterpret_cast<const vf*>(src + (a * 6 + bb) * plane));
#pragma unroll
      for (int p = 0; p < 4; ++p)
        if (kAT43[p][a] != 0.f)
#pragma unroll
          for (int bb = 0; bb < 6; ++bb) s[p][bb] = __builtin_elementwise_fma(vf(kAT43[p][a]), mr[bb], s[p][bb]);
    }
    const vf sc = d.scale ? *reinterpret_cast<const vf*>(d.scale + n) : vf(1.f);
    const vf sh = d.shift ? *reinterpret_cast<const vf*>(d.shift + n) : vf(0.f);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int oy = 4 * ty + p;
      if (oy >= d.Ho) break;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int ox = 4 * tx + qq;
        if (ox >= d.Wo) break;
        vf y = vf(0.f);
#pragma unroll
        for (int bb = 0; bb < 6; ++bb)
          if (kAT43[qq][bb] != 0.f) y = __builtin_elementwise_fma(vf(kAT43[qq][bb]), s[p][bb], y);
        const int64_t m = (b * d.Ho + oy) * d.Wo + ox;
        SP_BCHECK(m, (int64_t)d.N * d.Ho * d.Wo);
        y = __builtin_elementwise_fma(y, sc, sh);
        if (d.res1) y += *reinterpret_cast<const vf*>(d.res1 + m * d.ldr1 + n);
#pragma unroll
        for (int e = 0; e < VW; ++e) y[e] = act_apply(y[e], d.act);
        if (d.res2) y += *reinterpret_cast<const vf*>(d.res2 + m * d.ldr2 + n);
        *reinterpret_cast<vf*>(d.C + m * d.ldc + n) = y;
      }
    }
  }
}

// Channels per thread of the F(4×4) transforms (profiles/r2/wino43_vw_ab.json, same-box A/B): the
// output transform is 2-10 % faster on one channel per thread at every C2 shape (more waves in flight
// hide the strided M reads); the input transform gains from two on large maps and loses on small ones
// (below 2^18 tile × channel items: bs1/bs8 maps). The results are the same either way (per-channel
// arithmetic is identical). A tuning build (-DSP_TUNING_BUILD) lets SP_WINO43_VW=1|2 force one for such
// A/Bs; the product build reads no environment.
int wino43_forced_vw() {
#ifdef SP_TUNING_BUILD
  static const int forced = [] {
    const char* e = getenv("SP_WINO43_VW");
    const int v = e ? atoi(e) : 0;
    return v == 1 || v == 2 ? v : 0;
  }();
  return forced;
#else
  return 0;
#endif
}
int wino43_in_vw(int64_t items) {
  const int f = wino43_forced_vw();
  return f ? f : items < (int64_t(1) << 18) ? 1 : 2;
}
int wino43_out_vw() {
  const int f = wino43_forced_vw();
  return f ? f : 1;
}

int stream_grid(int64_t work) {
  int64_t g = (work + 255) / 256;
  const int64_t cap = (int64_t)g_num_cus * 16;
  return (int)(g < cap ? (g > 0 ? g : 1) : cap);
}

bool al16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

}  // namespace
}  // namespace sp

namespace sp {
namespace {

// Validation shared by the Winograd entry points (output tiles MT × MT: 2 for F(2×2,3×3), 4 for
// F(4×4,3×3); NC = (MT + 2)² components); fills th, tw, T. wt_wino may be null (the transform stages
// do not read it).
// Floats of the workspace that V occupies (M follows): NC·T·Cin fp32.
int64_t wino_v_floats(int nc, int64_t T, int cin) { return (int64_t)nc * T * cin; }

template <int MT>
int wino_check(const char* what, const sp_conv_desc* d, const uint16_t* wt_wino, int64_t wino_plane_stride,
               const float* work, int64_t work_elems, bool need_wt, int* th, int* tw, int64_t* T) {
  constexpr int NC = (MT + 2) * (MT + 2);
  SP_ARG_CHECK(d != nullptr && work != nullptr && (!need_wt || wt_wino != nullptr), "%s: null argument", what);
  SP_ARG_CHECK(d->A && d->C, "%s: null A/C", what);
  SP_ARG_CHECK(d->KH == 3 && d->KW == 3 && d->stride == 1 && d->pad == 1 && d->Ho == d->H && d->Wo == d->W,
               "%s: needs a 3x3 stride-1 pad-1 conv (KH=%d KW=%d stride=%d pad=%d)", what, d->KH, d->KW, d->stride,
               d->pad);
  SP_ARG_CHECK(d->N > 0 && d->H > 0 && d->W > 0, "%s: bad shape", what);
  SP_ARG_CHECK(d->Cin % 32 == 0 && d->Cout % 4 == 0 && d->Cout > 0,
               "%s: needs Cin %% 32 == 0, Cout %% 4 == 0 (Cin=%d Cout=%d)", what, d->Cin, d->Cout);
  SP_ARG_CHECK(d->precision == SP_PREC_F32X3 || d->precision == SP_PREC_BF16,
               "%s: precision %d (split or bf16 operands)", what, d->precision);
  SP_ARG_CHECK(!d->A2 && !d->row_scale && d->out_rows_per_group == 0 && !d->ln_gamma,
               "%s: A2 / row_scale / grouped rows / LayerNorm are not supported", what);
  const int planes = d->precision == SP_PREC_BF16 ? 1 : 3;
  SP_ARG_CHECK(!need_wt || planes == 1 || wino_plane_stride >= (int64_t)NC * d->Cout * d->Cin,
               "%s: wino_plane_stride %lld < %d*Cout*Cin", what, (long long)wino_plane_stride, NC);
  SP_ARG_CHECK(d->lda % 4 == 0 && d->ldc % 4 == 0 && al16(d->A) && al16(d->C) && (!need_wt || al16(wt_wino)) &&
                   (!need_wt || planes == 1 || wino_plane_stride % 8 == 0) &&
                   (!d->res1 || (d->ldr1 % 4 == 0 && al16(d->res1))) &&
                   (!d->res2 || (d->ldr2 % 4 == 0 && al16(d->res2))) && (!d->scale || al16(d->scale)) &&
                   (!d->shift || al16(d->shift)) && al16(work),
               "%s: operands must be 16-byte aligned with row strides %% 4 == 0", what);
  *th = (d->H + MT - 1) / MT;
  *tw = (d->W + MT - 1) / MT;
  *T = (int64_t)d->N * *th * *tw;
  SP_ARG_CHECK(*T < 0x7fffffff, "%s: %lld tiles", what, (long long)*T);
  const int64_t need = wino_v_floats(NC, *T, d->Cin) + (int64_t)NC * *T * d->Cout;
  SP_ARG_CHECK(work_elems >= need, "%s: workspace %lld < %lld elements", what, (long long)work_elems,
               (long long)need);
  return 0;
}

template <int MT>
int wino_input(const char* what, const sp_conv_desc* d, float* work, int64_t work_elems, void* stream) {
  constexpr int NC = (MT + 2) * (MT + 2);
  int th, tw;
  int64_t T;
  if (int rc = wino_check<MT>(what, d, nullptr, 0, work, work_elems, false, &th, &tw, &T)) return rc;
  if constexpr (MT == 2) {
    const int cin4 = d->Cin / 4;
    const int64_t pairs = (int64_t)d->N * th * ((tw + 1) / 2);
    hipLaunchKernelGGL(wino_in_f23_x2_kernel, dim3(stream_grid(pairs * cin4)), dim3(256), 0, as_stream(stream),
                       d->A, d->lda, d->H, d->W, cin4, th, tw, (int64_t)d->N, work, (int64_t)d->Cin);
  } else {
    const int64_t ts = d->Cin, cs = T * d->Cin;
    if (wino43_in_vw(T * d->Cin) == 1)
      hipLaunchKernelGGL(wino_in_f43_kernel<1>, dim3(stream_grid(T * d->Cin)), dim3(256), 0, as_stream(stream),
                         d->A, d->lda, d->H, d->W, d->Cin, th, tw, T, work, ts, cs);
    else
      hipLaunchKernelGGL(wino_in_f43_kernel<2>, dim3(stream_grid(T * d->Cin / 2)), dim3(256), 0, as_stream(stream),
                         d->A, d->lda, d->H, d->W, d->Cin / 2, th, tw, T, work, ts, cs);
  }
  return check_launch(what);
}

template <int MT>
int wino_gemm(const char* what, const sp_conv_desc* d, const uint16_t* wt_wino, int64_t wino_plane_stride,
              float* work, int64_t work_elems, void* stream) {
  constexpr int NC = (MT + 2) * (MT + 2);
  int th, tw;
  int64_t T;
  if (int rc = wino_check<MT>(what, d, wt_wino, wino_plane_stride, work, work_elems, true, &th, &tw, &T)) return rc;
  const int planes = d->precision == SP_PREC_BF16 ? 1 : 3;
  // the NC component GEMMs as one batched launch: M = T tiles, K = Cin, no epilogue
  ConvArgs g;
  memset(&g.d, 0, sizeof(g.d));
  const int64_t voff = wino_v_floats(NC, T, d->Cin);
  g.d.A = work;
  g.d.lda = d->Cin;
  g.d.N = 1;
  g.d.H = 1;
  g.d.W = (int32_t)T;
  g.d.Cin = d->Cin;
  g.d.KH = g.d.KW = 1;
  g.d.stride = 1;
  g.d.pad = 0;
  g.d.Ho = 1;
  g.d.Wo = (int32_t)T;
  g.d.Cout = d->Cout;
  g.d.C = work + voff;
  g.d.ldc = d->Cout;
  g.d.precision = d->precision;
  g.d.Wt_bf16 = wt_wino;
  g.d.wt_plane_stride = wino_plane_stride;
  g.M = T;
  g.K = d->Cin;
  g.HoWo = (int32_t)T;
  g.fast = 1;
  g.vec_epi = 1;
  g.splits = 1;
  g.ldp = d->Cout;
  g.partial = nullptr;
  g.batch = NC;
  g.bs_a = T * d->Cin;
  g.bs_w = (int64_t)d->Cout * d->Cin;
  g.bs_c = T * d->Cout;
  // tile: a forced LDS-DMA configuration (tuning), else the measured choice (tools/tune_wino.py): 64×64 (cfg
  // 14) when Cout is not a multiple of 128 or the batch is short (fewer than 12000 NC × T rows: the bs1 / bs8
  // maps, where the larger tiles leave CUs idle; 1.4x at bs1 40²×384, profiles/r2/tune_wino_f43_bs1.json,
  // tune_wino_x3_bs8_bs1.json); else the direct-store epilogue forms (cfg + 200, round 4,
  // profiles/r4/x3/tune_wino_f43_r4.json, whole-conv times at bs32 vs the round-3 choice): 128×128 k32 on
  // 16x16x32 MFMAs (247) for the wide batches from 400000 rows (80²×384: 1.162 vs 1.241 ms for cfg 44),
  // 128×128 k16 at four workgroups per CU (246) for Cout <= 256 (40²×256: 0.177 vs 0.184; 80²×128: 0.268 vs
  // 0.282), 128×128 k32 (245) otherwise (40²×384: 0.308 vs 0.327; 20²×512: 0.140 vs 0.150 for cfg 47).
  int cfg = forced_cfg();
  if (cfg < 0) {
    // short batches (the bs1 80² maps, 14400 rows; not the bs32 20² maps at 28800): 256×128 with eight 32×128
    // waves for Cout >= 256 (0.0395 vs 0.0535 ms for 245 at 80²×384), else 64×64 (0.0103 vs 0.0114 for 246 at
    // 80²×128; profiles/r5/bs1/tune_bs1_cross.json)
    if (d->Cout % 128 == 0 && T * NC >= 12000 && T * NC < 20000) cfg = d->Cout >= 256 ? 63 : 14;
    else if (d->Cout % 128 || T * NC < 12000) cfg = 14;
    else if (T * NC >= 400000 && d->Cout >= 384) cfg = 247;
    else if (d->Cout <= 256) cfg = 246;
    else cfg = 245;
  }
  const int rc = launch_glds_cfg(g, planes, cfg, as_stream(stream));
  if (rc == -2) {
    set_error("%s: tile configuration %d is not an LDS-DMA configuration", what, cfg);
    return -1;
  }
  return rc;
}

template <int MT>
int wino_output(const char* what, const sp_conv_desc* d, const float* work, int64_t work_elems, void* stream) {
  constexpr int NC = (MT + 2) * (MT + 2);
  int th, tw;
  int64_t T;
  if (int rc = wino_check<MT>(what, d, nullptr, 0, work, work_elems, false, &th, &tw, &T)) return rc;
  if constexpr (MT == 2) {
    const int cout4 = d->Cout / 4;
    hipLaunchKernelGGL(wino_out_f23_kernel, dim3(stream_grid(T * cout4)), dim3(256), 0, as_stream(stream),
                       work + wino_v_floats(NC, T, d->Cin), T, cout4, th, tw, *d);
  } else {
    const int64_t ts = d->Cout, cs = T * d->Cout;
    if (wino43_out_vw() == 1)
      hipLaunchKernelGGL(wino_out_f43_kernel<1>, dim3(stream_grid(T * d->Cout)), dim3(256), 0, as_stream(stream),
                         work + wino_v_floats(NC, T, d->Cin), T, d->Cout, th, tw, *d, ts, cs);
    else
      hipLaunchKernelGGL(wino_out_f43_kernel<2>, dim3(stream_grid(T * d->Cout / 2)), dim3(256), 0,
                         as_stream(stream), work + wino_v_floats(NC, T, d->Cin), T, d->Cout / 2, th, tw, *d, ts, cs);
  }
  return check_launch(what);
}

}  // namespace
}  // namespace sp

extern "C" int sp_winograd_f23_input(const sp_conv_desc* d, float* work, int64_t work_elems, void* stream) {
  return sp::wino_input<2>("sp_winograd_f23_input", d, work, work_elems, stream);
}

extern "C" int sp_winograd_f23_gemm(const sp_conv_desc* d, const uint16_t* wt_wino, int64_t wino_plane_stride,
                                    float* work, int64_t work_elems, void* stream) {
  return sp::wino_gemm<2>("sp_winograd_f23_gemm", d, wt_wino, wino_plane_stride, work, work_elems, stream);
}

extern "C" int sp_winograd_f23_output(const sp_conv_desc* d, const float* work, int64_t work_elems, void* stream) {
  return sp::wino_output<2>("sp_winograd_f23_output", d, work, work_elems, stream);
}

extern "C" int sp_conv3x3_winograd(const sp_conv_desc* d, const uint16_t* wt_wino, int64_t wino_plane_stride,
                                   float* work, int64_t work_elems, void* stream) {
  if (int rc = sp_winograd_f23_input(d, work, work_elems, stream)) return rc;
  if (int rc = sp_winograd_f23_gemm(d, wt_wino, wino_plane_stride, work, work_elems, stream)) return rc;
  return sp_winograd_f23_output(d, work, work_elems, stream);
}

extern "C" int sp_winograd_f43_input(const sp_conv_desc* d, float* work, int64_t work_elems, void* stream) {
  return sp::wino_input<4>("sp_winograd_f43_input", d, work, work_elems, stream);
}

extern "C" int sp_winograd_f43_gemm(const sp_conv_desc* d, const uint16_t* wt_wino, int64_t wino_plane_stride,
                                    float* work, int64_t work_elems, void* stream) {
  return sp::wino_gemm<4>("sp_winograd_f43_gemm", d, wt_wino, wino_plane_stride, work, work_elems, stream);
}

extern "C" int sp_winograd_f43_output(const sp_conv_desc* d, const float* work, int64_t work_elems, void* stream) {
  return sp::wino_output<4>("sp_winograd_f43_output", d, work, work_elems, stream);
}
