#!/bin/bash
# Round-4 x3 re-tune (GPU box, repo root): the C2 step's split-mode shapes with the direct-store epilogue
# forms (cfg + 200) beside the slab forms, from a fresh --detail of the current tree.
set -e
O=gpurun_out/w4
mkdir -p $O
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --latency-iters 0 --steps 5 --warmup 2 --detail $O/detail_c2.json > $O/bench_c2.log 2>&1
timeout -k 10 900 python -u tools/tune_conv.py $O/detail_c2.json --steps 5 --modes x3 --min-ms 0.1 \
  --cfgs=-,12,14,33,41,44,45,46,47,63,64,212,214,241,245,246,247,263,264 --out $O/tune_c2_x3.json > $O/tune_c2_x3.log 2>&1
