#!/bin/bash
# conv_x3s_kernel ablation builds (SP_X3S_ABL bit masks) into spotter_amd/_ablate/ for
# tools/conv_bench.py via SPOTTER_HIP_LIB (timing only; the results of these builds are wrong).
set -e
cd "$(dirname "$0")/.."
mkdir -p spotter_amd/_ablate
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -Xarch_host -ffp-contract=off -munsafe-fp-atomics -Iinclude"
OBJS=$(ls spotter_amd/_build/*.o | grep -v conv_mfma16)
for A in "$@"; do
  /opt/rocm/bin/hipcc $F -DSP_X3S_ABL=$A -c spotter_amd/csrc/conv_mfma16.hip -o spotter_amd/_ablate/x3s_$A.o &
done
wait
for A in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS spotter_amd/_ablate/x3s_$A.o -o spotter_amd/_ablate/libx3s_$A.so
done
