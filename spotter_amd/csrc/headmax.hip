// Query selection's score head of the bf16 variant in one pass: enc_outputs_class = enc_score_head(output_memory)
// (M2:1587-1593) and its per-anchor max over the classes (enc_outputs_class.max(-1).values, M2:1599), fused so
// the [B·S, C] logits never reach HBM: sp_conv2d + sp_rowmax wrote and re-read 2 × 688 MB of fp32 logits per
// C3 step only for the top-k key.
//
// The arithmetic is the bf16-mode GEMM's, element for element: v_mfma_f32_32x32x16_bf16 with A = the bf16 rows
// (lane l: row l & 31, k = 16s + 8(l >> 5) .. +8) and B = the bf16 weights (column l & 31, same k), k in 16-deep
// steps from 0 upwards, + bias by fmaf(acc, 1, bias) as the GEMM epilogue does, then fmaxf over the classes —
// so the row maxima equal sp_rowmax of the GEMM's logits bit for bit (tests/test_gpu_kernels.py).
//
// Layout: the weights (N ≤ 96 classes × K = 256, zero rows up to 96) sit in LDS for the whole workgroup, 16-byte
// chunks swizzled by row (chunk c of row r at c ^ (r & 15)) so a wave's 32 rows of one k-chunk fall on distinct
// bank groups; each wave owns 32 anchors per block and walks the blocks of a persistent grid (the weights are
// staged once per workgroup, not once per 128 anchors).
#include "common.h"

namespace sp {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int HM_NP = 96;     // class columns staged (3 blocks of 32)

template <int KC>  // K / 8: 16-byte chunks per row
__global__ __launch_bounds__(256, 2) void linear_rowmax_bf16_kernel(const uint16_t* __restrict__ a, int64_t lda,
                                                                     const uint16_t* __restrict__ w,
                                                                     const float* __restrict__ bias, int rows, int n,
                                                                     float* __restrict__ out) {
  __shared__ uint4 wl[HM_NP * KC];
  __shared__ float red[4][16][2][33];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int r = lane & 31, h = lane >> 5;
  for (int i = tid; i < HM_NP * KC; i += 256) {
    const int row = i / KC, c = i - row * KC;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (row < n) v = *reinterpret_cast<const uint4*>(w + (int64_t)row * KC * 8 + c * 8);
    wl[row * KC + (c ^ (row & 15))] = v;
  }
  float bv[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) bv[j] = j * 32 + r < n ? bias[j * 32 + r] : 0.f;
  __syncthreads();
  const int nblk = (rows + 127) / 128;
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t rb = (int64_t)blk * 128 + wave * 32;
    const int64_t row = rb + r < rows ? rb + r : rows - 1;
    const uint4* ar = reinterpret_cast<const uint4*>(a + row * lda);
    SP_BCHECK(row, rows);
    uint4 af[KC / 2];
#pragma unroll
    for (int s = 0; s < KC / 2; ++s) af[s] = ar[2 * s + h];
    f32x16 acc[3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[j][q] = 0.f;
#pragma unroll
    for (int s = 0; s < KC / 2; ++s) {
      const bf16x8 fa = __builtin_bit_cast(bf16x8, af[s]);
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int brow = j * 32 + r;
        const bf16x8 fb = __builtin_bit_cast(bf16x8, wl[brow * KC + ((2 * s + h) ^ (brow & 15))]);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[j], 0, 0, 0);
      }
    }
    // lane (r, h), element q: row (q & 3) + 8 (q >> 2) + 4 h of the 32, class j·32 + r
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      float m = -INFINITY;
#pragma unroll
      for (int j = 0; j < 3; ++j)
        if (j * 32 + r < n) m = fmaxf(m, fmaf(acc[j][q], 1.0f, bv[j]));
      red[wave][q][h][r] = m;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (lane < 32) {
      const int t = lane;  // row t of the 32: q = (t & 3) | ((t >> 3) << 2), h = (t >> 2) & 1
      const int q = (t & 3) | ((t >> 3) << 2), hh = (t >> 2) & 1;
      float m = -INFINITY;
#pragma unroll
      for (int i = 0; i < 32; ++i) m = fmaxf(m, red[wave][q][hh][i]);
      if (rb + t < rows) out[rb + t] = m;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
}

}  // namespace
}  // namespace sp

extern "C" int sp_linear_rowmax_bf16(const uint16_t* a, int64_t lda, const uint16_t* w, const float* bias, int rows,
                                     int n, int k, float* out, void* stream) {
  using namespace sp;
  SP_ARG_CHECK(a && w && bias && out && rows > 0 && n > 0 && n <= HM_NP && k == 256,
               "sp_linear_rowmax_bf16: bad args (n <= %d, k = 256)", HM_NP);
  SP_ARG_CHECK(lda >= k && lda % 8 == 0 && ((uintptr_t)a & 15) == 0 && ((uintptr_t)w & 15) == 0,
               "sp_linear_rowmax_bf16: 16-byte aligned rows, lda %% 8 == 0");
  const int nblk = (rows + 127) / 128;
  const int grid = nblk < 2 * g_num_cus ? nblk : 2 * g_num_cus;  // two workgroups per CU (66 KB of LDS each)
  hipLaunchKernelGGL(linear_rowmax_bf16_kernel<32>, dim3(grid), dim3(256), 0, as_stream(stream), a, lda, w, bias,
                     rows, n, out);
  return check_launch("sp_linear_rowmax_bf16");
}
