#!/bin/bash
# Diagnostic library builds into spotter_amd/_diag/ (not the product): tools/build_diag.sh <name> <-D flags...>
# e.g. tools/build_diag.sh stamp -DSP_GLDS_STAMP=1 → spotter_amd/_diag/libspotter_stamp.so (conv_glds.hip rebuilt
# with the flags, every other object from spotter_amd/_build/). Use with SPOTTER_HIP_LIB=<that .so>.
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p spotter_amd/_diag
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -Xarch_host -ffp-contract=off -munsafe-fp-atomics -Iinclude"
OBJS=$(ls spotter_amd/_build/*.o | grep -v conv_glds)  # the diag unit instantiates every part itself
/opt/rocm/bin/hipcc $F -DSP_GLDS_ONE_UNIT=1 "$@" -c spotter_amd/csrc/conv_glds.hip -o spotter_amd/_diag/conv_glds_$NAME.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS spotter_amd/_diag/conv_glds_$NAME.o -o spotter_amd/_diag/libspotter_$NAME.so
echo built spotter_amd/_diag/libspotter_$NAME.so
