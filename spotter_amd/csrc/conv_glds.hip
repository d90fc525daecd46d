// LDS-DMA implicit-GEMM kernels on bf16-operand MFMA (x3 split / bf16): the dispatcher of the tile
// configurations 11-65 of launch_mfma16 (conv_mfma16.hip). The kernels live in conv_glds.h and are
// instantiated across conv_glds_p<k>.hip; a diagnostic build (tools/build_diag.sh: -DSP_GLDS_ONE_UNIT plus
// -DSP_GLDS_STAMP or -DSP_ABLATE=n) instantiates them all here instead.
#include "conv_glds.h"

namespace sp {

#if SP_GLDS_STAMP || SP_GLDS_ONE_UNIT
namespace {
int glds_part_k(int k, const ConvArgs& a, int planes, int cfg, hipStream_t s, int epv) {
  switch (k) {
    case 0: return glds_part<0>(a, planes, cfg, s, epv);
    case 1: return glds_part<1>(a, planes, cfg, s, epv);
    case 2: return glds_part<2>(a, planes, cfg, s, epv);
    case 3: return glds_part<3>(a, planes, cfg, s, epv);
    case 4: return glds_part<4>(a, planes, cfg, s, epv);
    default: return glds_part<5>(a, planes, cfg, s, epv);
  }
}
}  // namespace
#else
int launch_glds_part0(const ConvArgs& a, int planes, int cfg, hipStream_t s, int epv);
int launch_glds_part1(const ConvArgs& a, int planes, int cfg, hipStream_t s, int epv);
int launch_glds_part2(const ConvArgs& a, int planes, int cfg, hipStream_t s, int epv);
int launch_glds_part3(const ConvArgs& a, int planes, int cfg, hipStream_t s, int epv);
int launch_glds_part4(const ConvArgs& a, int planes, int cfg, hipStream_t s, int epv);
int launch_glds_part5(const ConvArgs& a, int planes, int cfg, hipStream_t s, int epv);
namespace {
int glds_part_k(int k, const ConvArgs& a, int planes, int cfg, hipStream_t s, int epv) {
  switch (k) {
    case 0: return launch_glds_part0(a, planes, cfg, s, epv);
    case 1: return launch_glds_part1(a, planes, cfg, s, epv);
    case 2: return launch_glds_part2(a, planes, cfg, s, epv);
    case 3: return launch_glds_part3(a, planes, cfg, s, epv);
    case 4: return launch_glds_part4(a, planes, cfg, s, epv);
    default: return launch_glds_part5(a, planes, cfg, s, epv);
  }
}
}  // namespace
#endif
static_assert(kGldsParts == 6, "one conv_glds_p<k>.hip per part");

// The LDS-DMA configurations (see launch_mfma16); -2 when cfg is not one of them. cfg + 100: the same tile
// with the LDS-DMA residual epilogue (epilogue_tile_rd) on the split mode's 1×1 path.
int launch_glds_cfg(const ConvArgs& a, int planes, int cfg, hipStream_t s) {
  // cfg + 100: the slab epilogue (variants 2 / 3); cfg + 200: its direct-store form (variant 4) where it applies
  const int epv = cfg >= 200 ? 4 : cfg >= 100 ? 2 : 1;
  cfg %= 100;
  if (a.d.A2 || cfg < 11 || cfg > 65) return -2;
  return glds_part_k(cfg % kGldsParts, a, planes, cfg, s, epv);
}

}  // namespace sp

#if SP_GLDS_STAMP
extern "C" int sp_debug_glds_stamps(void* dst) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(sp::g_glds_stamps), sizeof(sp::g_glds_stamps));
}
#endif
