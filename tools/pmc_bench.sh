#!/bin/bash
# HBM traffic of the bench's kernels from PMC counters — run on the GPU box from the repo root:
#   tools/pmc_bench.sh <outdir> [bench.py args...]
# Two separate passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950), each with
# --kernel-trace only, then tools/pmc_reduce.py folds them into profiles/pmc_traffic.json.
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --latency-iters 0 --no-events $*"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o pmc \
  -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o pmc \
  -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1
python3 tools/pmc_reduce.py "$OUT" $ARGS > "$OUT/traffic.json"; cat "$OUT/traffic.json"
