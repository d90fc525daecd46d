// Error state, device init and ABI version of libspotter_hip.
#include "common.h"

namespace sp {

static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = 0; }

}  // namespace sp

extern "C" int sp_abi_version(void) { return SP_ABI_VERSION; }

namespace sp {
namespace {
struct BoundsUnit {
  const char* unit;
  int (*read)(BoundsLog*, int);
};
// function-local storage: the registrations run from other units' static initialisers
BoundsUnit* bounds_units(int** count) {
  static BoundsUnit units[64];
  static int n = 0;
  *count = &n;
  return units;
}
}  // namespace

int bounds_register(const char* unit, int (*read)(BoundsLog*, int)) {
  int* n;
  BoundsUnit* u = bounds_units(&n);
  if (*n < 64) u[(*n)++] = {unit, read};
  return *n;
}
}  // namespace sp

extern "C" int sp_build_flags(void) {
  return (sp::conv_gemm_has_fused_ln() ? SP_BUILD_FUSED_LN : 0) | (SP_BOUNDS ? SP_BUILD_BOUNDS : 0);
}

extern "C" int64_t sp_bounds_report(char* buf, int64_t cap) {
#if SP_BOUNDS
  int* n;
  sp::BoundsUnit* u = sp::bounds_units(&n);
  int64_t total = 0, used = 0;
  if (buf && cap > 0) buf[0] = 0;
  for (int i = 0; i < *n; ++i) {
    sp::BoundsLog lg;
    if (u[i].read(&lg, 1) != 0) {
      sp::set_error("sp_bounds_report: reading the log of %s failed", u[i].unit);
      return -2;
    }
    total += lg.hits;
    if (lg.hits && buf && used < cap) {
      const int w = snprintf(buf + used, (size_t)(cap - used), "%s:%d hits=%u index=%lld extent=%lld\n",
                             u[i].unit, lg.line, lg.hits, lg.index, lg.extent);
      if (w > 0) used += w;
    }
  }
  return total;
#else
  (void)buf;
  (void)cap;
  sp::set_error("sp_bounds_report: not a bounds-check build (python -m spotter_amd.build_ext --bounds)");
  return -1;
#endif
}

extern "C" const char* sp_last_error(void) { return sp::g_err; }

namespace sp {
int g_num_cus = 256;
}

extern "C" int sp_device_init(int device) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    sp::set_error("hipSetDevice(%d): %s", device, hipGetErrorString(e));
    return (int)e;
  }
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, device);
  if (e != hipSuccess) {
    sp::set_error("hipGetDeviceProperties: %s", hipGetErrorString(e));
    return (int)e;
  }
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    sp::set_error("libspotter_hip is built for gfx950 (MI355X); device %d is %s", device,
                  prop.gcnArchName);
    return -2;
  }
  sp::g_num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  return 0;
}

extern "C" int sp_shutdown(void) {
  sp::free_coeff_cache();
  return 0;
}
