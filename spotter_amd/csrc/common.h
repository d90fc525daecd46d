// Shared helpers for the libspotter_hip kernels (gfx950 / CDNA4 only).
#pragma once

// Bounds-check diagnostic build ("HIP kernels get bounds-checked debug builds"):
// python -m spotter_amd.build_ext --bounds compiles every unit with -DSP_BOUNDS=1 into
// spotter_amd/_bounds/libspotter_bounds.so. SP_BCHECK(index, extent) then guards the global index sites of
// the kernels: a violation is counted in its translation unit's device log (the first one's line, index and
// extent kept) instead of trapping, so one GPU run reports every site; sp_bounds_report() collects and resets
// the logs. The product library compiles SP_BCHECK to nothing.
#ifndef SP_BOUNDS
#define SP_BOUNDS 0
#endif

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

// A translation unit's bounds log (SP_BOUNDS builds): violations, and the first one's source line, index, extent.
struct BoundsLog {
  unsigned int hits;
  int line;
  long long index, extent;
};
// registers a unit's log reader (runtime.hip; called from static initialisers of SP_BOUNDS builds)
int bounds_register(const char* unit, int (*read)(BoundsLog* out, int reset));
// what the library was compiled with (sp_build_flags): conv_gemm.hip's fused-LayerNorm tiles
bool conv_gemm_has_fused_ln();
// msda.hip's tuning hook (sp_set_tuning SP_TUNE_MSDA_GENERIC)
int msda_generic();
void set_msda_generic(int v);

#if SP_BOUNDS
namespace {
__device__ BoundsLog g_bounds_log;

__device__ __noinline__ void bounds_hit(int line, long long i, long long n) {
  if (atomicAdd(&g_bounds_log.hits, 1u) == 0u) {
    g_bounds_log.line = line;
    g_bounds_log.index = i;
    g_bounds_log.extent = n;
  }
}

int bounds_read(BoundsLog* out, int reset) {
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bounds_log), sizeof(BoundsLog)) != hipSuccess)
    return -1;
  if (reset) {
    const BoundsLog zero = {0u, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_bounds_log), &zero, sizeof(BoundsLog)) != hipSuccess) return -1;
  }
  return 0;
}

[[maybe_unused]] const int g_bounds_registered = bounds_register(__BASE_FILE__, &bounds_read);
}  // namespace
#define SP_BCHECK(idx, ext)                                                  \
  do {                                                                       \
    const long long sp_bi_ = (long long)(idx), sp_bn_ = (long long)(ext);    \
    if (sp_bi_ < 0 || sp_bi_ >= sp_bn_) ::sp::bounds_hit(__LINE__, sp_bi_, sp_bn_); \
  } while (0)
#else
#define SP_BCHECK(idx, ext) \
  do {                      \
  } while (0)
#endif

}  // namespace sp

#define SP_ARG_CHECK(cond, ...)      \
  do {                               \
    if (!(cond)) {                   \
      ::sp::set_error(__VA_ARGS__);  \
      return -1;                     \
    }                                \
  } while (0)
