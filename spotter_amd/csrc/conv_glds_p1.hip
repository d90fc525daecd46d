// One part of the LDS-DMA tile configurations (conv_glds.h: ids with id % 6 == 1), compiled as its own
// translation unit so the build runs the parts in parallel.
#include "conv_glds.h"

#if !(SP_GLDS_STAMP || SP_GLDS_ONE_UNIT)
namespace sp {
int launch_glds_part1(const ConvArgs& a, int planes, int cfg, hipStream_t s, int epv) {
  return glds_part<1>(a, planes, cfg, s, epv);
}
}  // namespace sp
#endif
