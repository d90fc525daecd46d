#!/bin/bash
# One GPU-box measurement pass over the current tree — run from the repo root on the GPU box:
#   tools/gpu_round.sh <tag>
# 1. pytest -m gpu (parity), 2. the default bench line (CPU baseline + p50 latency included),
# 3. rocprofv3 --kernel-trace --stats of the same bench (kernel averages to cross-check the HIP-event
# roofline), 4. the PMC HBM-traffic passes (tools/pmc_bench.sh). Every GPU step has its own time
# limit and the steps are chained, so the first failure ends the script.
set -euo pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/gpu_tests.log" 2>&1
tail -3 "$OUT/gpu_tests.log"
timeout -k 10 420 python3 -u bench.py > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench \
  -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 > "$OUT/prof.log" 2>&1
python3 tools/stats_classes.py "$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)" \
  --csv-out "$OUT/kernel_stats.csv" > "$OUT/kernel_classes.json"
bash tools/pmc_bench.sh "$OUT/pmc"
echo "gpu_round $TAG done"
