#!/bin/bash
# 16x16x32 variants: correctness, then every x3 shape of the bs32 step re-tuned over all split configurations
set -euo pipefail
OUT=gpurun_out/${1:-m16}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q -k "47 or 49 or 65" --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -1 "$OUT/tests.log"
timeout -k 10 900 python3 -u tools/tune_conv.py profiles/r2/conv_detail_fp32x3_r2.json --modes x3 --min-ms 0.02 --out "$OUT/tune.json" --reps 8 > "$OUT/tune.log" 2>&1
tail -1 "$OUT/tune.log"
