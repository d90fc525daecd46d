#!/bin/bash
# Builds libspotter_hip variants with conv_glds_kernel ablations (SP_ABLATE=1 no in-loop DMA,
# 2 no fp32 split, 3 no MFMA) into spotter_amd/_ablate/ for tools/conv_bench.py via SPOTTER_HIP_LIB.
set -e
cd "$(dirname "$0")/.."
mkdir -p spotter_amd/_ablate
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -Xarch_host -ffp-contract=off -munsafe-fp-atomics -Iinclude"
OBJS=$(ls spotter_amd/_build/*.o | grep -v conv_mfma16)
for A in 1 2 3; do
  /opt/rocm/bin/hipcc $F -DSP_ABLATE=$A -c spotter_amd/csrc/conv_mfma16.hip -o spotter_amd/_ablate/m16_$A.o &
done
wait
for A in 1 2 3; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS spotter_amd/_ablate/m16_$A.o -o spotter_amd/_ablate/lib_$A.so
done
