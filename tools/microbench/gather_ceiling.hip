// Gather ceiling for MSDA's access pattern (tools only, not the product).
//
// msda_vec_kernel (spotter_amd/csrc/msda.hip) samples, per query wave, 8 heads x L*P points x 4 bilinear
// corners; each corner is one 16-byte (fp32) or 8-byte (bf16) load per lane, the 8 lanes of a head reading
// one contiguous 128-byte (fp32) / 64-byte (bf16) row segment of the value map [B*S, ld]. This kernel issues
// exactly that address stream with uniformly random sampling locations (no offsets / logits / softmax reads,
// no output beyond one float per wave), the grid remapped XCD-major as msda does, so its rate is what
// random row-segment gathers from a map of this size sustain on this chip: the ceiling the MSDA kernel's
// gather rate is judged against.
//   NPT: sampling points whose 4 corners are issued before the first FMA (1, 4 = one level, 12 = all).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 ld4(const uint16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(__builtin_bit_cast(float, u.x << 16), __builtin_bit_cast(float, u.x & 0xffff0000u),
                     __builtin_bit_cast(float, u.y << 16), __builtin_bit_cast(float, u.y & 0xffff0000u));
}

struct Levels { int h[3], w[3], start[3]; };

template <typename VT, int NPT>
__global__ __launch_bounds__(256) void gather_kernel(const VT* __restrict__ value, int64_t ld, int S, int Q,
                                                     int64_t rows, Levels lv, float* __restrict__ out) {
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int64_t row = (int64_t)wg * 4 + (threadIdx.x >> 6);  // one query per wave
  if (row >= rows) return;
  const int t = threadIdx.x & 63, h = t >> 3, c = (t & 7) * 4;
  const int b = (int)(row / Q);
  const VT* vb = value + (int64_t)b * S * ld + h * 32 + c;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  constexpr int LP = 12;
#pragma unroll
  for (int g = 0; g < LP; g += NPT) {
    float4 v[NPT][4];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int i = g + j, l = i >> 2;
      const uint32_t r = mix((uint32_t)(row * 97 + h * 13 + i) * 0x9e3779b9u);
      const int W = lv.w[l], H = lv.h[l];
      const int x = (int)((r & 0xffff) * (uint32_t)(W - 1) >> 16), y = (int)((r >> 16) * (uint32_t)(H - 1) >> 16);
      const VT* p = vb + (int64_t)(lv.start[l] + y * W + x) * ld;
      v[j][0] = ld4(p);
      v[j][1] = ld4(p + ld);
      v[j][2] = ld4(p + (int64_t)W * ld);
      v[j][3] = ld4(p + (int64_t)(W + 1) * ld);
    }
#pragma unroll
    for (int j = 0; j < NPT; ++j)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float wk = 0.25f + 0.01f * k;
        acc.x += v[j][k].x * wk; acc.y += v[j][k].y * wk; acc.z += v[j][k].z * wk; acc.w += v[j][k].w * wk;
      }
  }
  const float s = acc.x + acc.y + acc.z + acc.w;
  if (s == 12345.678f) out[row] = s;  // keeps the loads live; never true for the benchmark's data
}

// the same bytes streamed once, contiguously (float4 per lane): the dense comparison
__global__ __launch_bounds__(256) void stream_kernel(const float4* __restrict__ p, int64_t n4, float* out) {
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 v = p[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.678f) out[0] = acc;
}

template <typename VT>
void launch(int npt, const void* value, int64_t ld, int S, int Q, int64_t rows, Levels lv, float* out,
            hipStream_t st) {
  const dim3 grid((unsigned)((rows + 3) / 4)), blk(256);
  const VT* v = (const VT*)value;
  if (npt == 1) hipLaunchKernelGGL((gather_kernel<VT, 1>), grid, blk, 0, st, v, ld, S, Q, rows, lv, out);
  else if (npt == 4) hipLaunchKernelGGL((gather_kernel<VT, 4>), grid, blk, 0, st, v, ld, S, Q, rows, lv, out);
  else hipLaunchKernelGGL((gather_kernel<VT, 12>), grid, blk, 0, st, v, ld, S, Q, rows, lv, out);
}

}  // namespace

// bf16: value is uint16 bit patterns. Levels: 80x80, 40x40, 20x20 (S = 8400) at 640^2, x2 each at 1280^2.
extern "C" int gather_ceiling(int bf16, int npt, const void* value, int64_t ld, int S, int Q, int B, int scale,
                              float* out, void* stream) {
  Levels lv;
  int start = 0;
  for (int l = 0; l < 3; ++l) {
    lv.h[l] = lv.w[l] = (80 >> l) * scale;
    lv.start[l] = start;
    start += lv.h[l] * lv.w[l];
  }
  if (start != S || (npt != 1 && npt != 4 && npt != 12)) return -1;
  const hipStream_t st = (hipStream_t)stream;
  if (bf16) launch<uint16_t>(npt, value, ld, S, Q, (int64_t)B * Q, lv, out, st);
  else launch<float>(npt, value, ld, S, Q, (int64_t)B * Q, lv, out, st);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int stream_read(const void* p, int64_t bytes, float* out, void* stream) {
  hipLaunchKernelGGL(stream_kernel, dim3(4096), dim3(256), 0, (hipStream_t)stream, (const float4*)p, bytes / 16, out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
