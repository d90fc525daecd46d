#!/bin/bash
# per-shape timings + tile tuner for the bf16 C2 variant and C5 (R101vd 1280² bs8 fp32) (GPU box)
set -euo pipefail
OUT=gpurun_out/${1:-tune_more}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u bench.py --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 --detail "$OUT/detail_bf16.json" > "$OUT/bench_bf16.log" 2>&1
timeout -k 10 600 python3 -u tools/tune_conv.py "$OUT/detail_bf16.json" --steps 5 --out "$OUT/tune_bf16.json" --reps 6 > "$OUT/tune_bf16.log" 2>&1
tail -1 "$OUT/tune_bf16.log"
timeout -k 10 300 python3 -u bench.py --size 1280 --batch 8 --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 --detail "$OUT/detail_c5.json" > "$OUT/bench_c5.log" 2>&1
timeout -k 10 600 python3 -u tools/tune_conv.py "$OUT/detail_c5.json" --steps 5 --out "$OUT/tune_c5.json" --reps 6 > "$OUT/tune_c5.log" 2>&1
tail -1 "$OUT/tune_c5.log"
