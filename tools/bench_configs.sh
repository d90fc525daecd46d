#!/bin/bash
# The non-default BASELINE.json configurations as bench lines (GPU box, repo root):
#   tools/bench_configs.sh <tag>
# C3: R18vd bf16 bs256; C5: R101vd 1280² bs8 (fp32 parity path); the bf16 variant of C2.
# No CPU baseline / latency legs (those belong to the default C2 line).
set -euo pipefail
OUT=gpurun_out/${1:-cfg}
mkdir -p "$OUT"
B="python3 -u bench.py --no-cpu-baseline --latency-iters 0"
timeout -k 10 300 $B --preset r18vd --precision bf16 --batch 256 > "$OUT/c3_r18vd_bf16_bs256.log" 2>&1
tail -1 "$OUT/c3_r18vd_bf16_bs256.log" | cut -c1-200
timeout -k 10 300 $B --size 1280 --batch 8 > "$OUT/c5_r101vd_1280_bs8.log" 2>&1
tail -1 "$OUT/c5_r101vd_1280_bs8.log" | cut -c1-200
timeout -k 10 300 $B --precision bf16 > "$OUT/c2_bf16.log" 2>&1
tail -1 "$OUT/c2_bf16.log" | cut -c1-200
