#!/bin/bash
# f32-mode layers timed under both fp32-accurate operand modes (Engine._pick's choice)
set -euo pipefail
OUT=gpurun_out/${1:-cross}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u tools/tune_conv.py profiles/r2/conv_detail_fp32x3_r2.json --modes f32 --cross --min-ms 0.01 --out "$OUT/tune.json" --reps 10 > "$OUT/tune.log" 2>&1
tail -1 "$OUT/tune.log"
