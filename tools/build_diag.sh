#!/bin/bash
# Diagnostic library builds into spotter_amd/_diag/ (not the product): tools/build_diag.sh <name> <-D flags...>
# e.g. tools/build_diag.sh stamp -DSP_GLDS_STAMP=1 → spotter_amd/_diag/libspotter_stamp.so (conv_glds.hip rebuilt
# with the flags, every other object from spotter_amd/_build/). Use with SPOTTER_HIP_LIB=<that .so>.
# UNIT=stem rebuilds csrc/stem.hip instead (e.g. UNIT=stem tools/build_diag.sh c64abl1 -DSP_C64_ABL=1).
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p spotter_amd/_diag
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -Xarch_host -ffp-contract=off -munsafe-fp-atomics -Iinclude"
UNIT=${UNIT:-conv_glds}
if [ "$UNIT" = conv_glds ]; then
  OBJS=$(ls spotter_amd/_build/*.o | grep -v conv_glds)  # the diag unit instantiates every part itself
  F="$F -DSP_GLDS_ONE_UNIT=1"
else
  OBJS=$(ls spotter_amd/_build/*.o | grep -v "/$UNIT\.o$")
fi
/opt/rocm/bin/hipcc $F "$@" -c spotter_amd/csrc/$UNIT.hip -o spotter_amd/_diag/${UNIT}_$NAME.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS spotter_amd/_diag/${UNIT}_$NAME.o -o spotter_amd/_diag/libspotter_$NAME.so
echo built spotter_amd/_diag/libspotter_$NAME.so
