#!/bin/bash
# x3 tile-config sweep on the dominant bs32 shapes (GPU box, repo root): tools/r2_cfg.sh <tag> <cfgs> [shapes]
set -euo pipefail
OUT=gpurun_out/${1:-cfg}
mkdir -p "$OUT"
timeout -k 10 400 python3 -u tools/conv_bench.py --prec f32x3 --cfgs="$2" --shapes "${3:-0,1,2,3,4,5,6}" --reps 10 > "$OUT/sweep.jsonl" 2>&1
cat "$OUT/sweep.jsonl" | cut -c1-160
