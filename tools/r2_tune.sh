#!/bin/bash
# per-shape timings of the default bench step, then the tile tuner over those shapes (GPU box)
set -euo pipefail
OUT=gpurun_out/${1:-tune}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --latency-iters 0 --detail "$OUT/detail.json" > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log" | cut -c1-200
timeout -k 10 900 python3 -u tools/tune_conv.py "$OUT/detail.json" --out "$OUT/tune.json" --reps 8 > "$OUT/tune.log" 2>&1
tail -1 "$OUT/tune.log"
