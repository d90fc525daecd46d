#!/bin/bash
# quick GPU check: full gpu tests + a bench line without the CPU baseline / latency legs
set -euo pipefail
TAG=${1:-q}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --latency-iters 0 ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log"
