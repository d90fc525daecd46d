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
