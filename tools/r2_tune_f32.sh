#!/bin/bash
set -euo pipefail
OUT=gpurun_out/${1:-tune_f32}
mkdir -p "$OUT"
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_kernels.py -x -q -k "every_tile_config" --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -1 "$OUT/tests.log"
timeout -k 10 600 python3 -u tools/tune_conv.py profiles/r2/conv_detail_fp32x3_r2.json --modes f32 --min-ms 0.01 --out "$OUT/tune.json" --reps 10 > "$OUT/tune.log" 2>&1
tail -1 "$OUT/tune.log"
