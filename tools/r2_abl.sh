#!/bin/bash
# conv_x3s ablation timings (tools/build_x3s_ablate.sh builds): tools/r2_abl.sh <tag> <cfg> <shapes> <abl...>
set -euo pipefail
OUT=gpurun_out/${1}; CFG=$2; SH=$3; shift 3
mkdir -p "$OUT"
timeout -k 10 120 python3 -u tools/conv_bench.py --prec f32x3 --cfgs=$CFG --shapes $SH --reps 10 > "$OUT/base.jsonl" 2>&1
for A in "$@"; do
  SPOTTER_HIP_LIB=spotter_amd/_ablate/libx3s_$A.so timeout -k 10 120 python3 -u tools/conv_bench.py --prec f32x3 --cfgs=$CFG --shapes $SH --reps 10 > "$OUT/abl_$A.jsonl" 2>&1
done
for f in "$OUT"/*.jsonl; do echo "$f"; grep shape "$f" | cut -c1-120; done
