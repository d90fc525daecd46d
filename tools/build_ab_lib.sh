#!/bin/bash
# An A/B library: the product objects with the listed units recompiled under extra defines, linked to _ab/.
#   tools/build_ab_lib.sh "<defines>" unit...     e.g. tools/build_ab_lib.sh "-DSP_EPI16_PAD=0" conv_glds_p0 ...
# Run bench / conv_bench against it with SPOTTER_HIP_LIB=_ab/libspotter_hip.so.
set -euo pipefail
DEF=$1; shift
mkdir -p _ab/obj
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -Xarch_host -ffp-contract=off -munsafe-fp-atomics -Iinclude"
objs=()
for o in spotter_amd/_build/*.o; do
  u=$(basename $o .o)
  if printf '%s\n' "$@" | grep -qx "$u"; then
    /opt/rocm/bin/hipcc $FLAGS $DEF -c spotter_amd/csrc/$u.hip -o _ab/obj/$u.o &
    objs+=(_ab/obj/$u.o)
  else
    objs+=($o)
  fi
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o _ab/libspotter_hip.so
echo built _ab/libspotter_hip.so
