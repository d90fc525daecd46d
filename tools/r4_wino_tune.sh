#!/bin/bash
# Round-4 (GPU box, repo root): the Winograd component GEMM's tiles with the direct-store epilogue forms, then
# the C2 line on the re-tuned table.
set -e
O=gpurun_out/w5
mkdir -p $O
timeout -k 10 600 python -u tools/tune_wino.py --m 4 --reps 10 --cfgs 14,44,45,46,47,63,64,214,244,245,246,247,263,264 \
  --out $O/tune_wino_f43_r4.json > $O/tune_wino.log 2>&1
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --latency-iters 0 > $O/bench_c2.log 2>&1
