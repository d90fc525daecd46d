#!/bin/bash
# C3 (R18vd bf16 bs256) per-shape timings + tile tuner (GPU box)
set -euo pipefail
OUT=gpurun_out/${1:-tune_c3}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u bench.py --preset r18vd --precision bf16 --batch 256 --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 --detail "$OUT/detail.json" > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log" | cut -c1-200
timeout -k 10 900 python3 -u tools/tune_conv.py "$OUT/detail.json" --steps 5 --out "$OUT/tune.json" --reps 6 > "$OUT/tune.log" 2>&1
tail -1 "$OUT/tune.log"
