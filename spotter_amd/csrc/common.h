// Shared helpers for the libspotter_hip kernels (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "../../include/spotter_hip.h"

namespace sp {

void set_error(const char* fmt, ...);
void clear_error();
void free_coeff_cache();

// Returns 0 after a successful async launch, else the hipError_t (and records it).
inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return static_cast<int>(e);
  }
  return 0;
}

// compute units of the device sp_device_init selected (MI355X: 256); sizes persistent grids
extern int g_num_cus;

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// torch.sigmoid on fp32: 1 / (1 + exp(-x))
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

}  // namespace sp

#define SP_ARG_CHECK(cond, ...)      \
  do {                               \
    if (!(cond)) {                   \
      ::sp::set_error(__VA_ARGS__);  \
      return -1;                     \
    }                                \
  } while (0)
