#!/bin/bash
# Builds libspotter_hip variants with conv_glds_kernel ablations (SP_ABLATE=1 no in-loop DMA, 2 no fp32 split,
# 3 no MFMA; results deliberately wrong, timing only) into spotter_amd/_diag/ via tools/build_diag.sh;
# use with SPOTTER_HIP_LIB=spotter_amd/_diag/libspotter_ablate<n>.so.
set -e
cd "$(dirname "$0")/.."
for A in 1 2 3; do bash tools/build_diag.sh ablate$A -DSP_ABLATE=$A; done
