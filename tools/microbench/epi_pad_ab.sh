#!/bin/bash
# A/B of the padded bf16 slab epilogue (product) against _ab/libspotter_hip.so (built with -DSP_EPI16_PAD=0 by
# tools/build_ab_lib.sh): conv_bench on the bf16-row shapes, then the C3 bench line, alternating libraries.
set -euo pipefail
OUT=${1:-gpurun_out/epipad}; mkdir -p $OUT
for r in 1 2; do
  for L in product ab; do
    if [ $L = ab ]; then export SPOTTER_HIP_LIB=_ab/libspotter_hip.so; else unset SPOTTER_HIP_LIB; fi
    timeout -k 10 200 python3 -u tools/conv_bench.py --prec bf16rows --shapes 31,39,28,29,30,37 --reps 10 > $OUT/conv_${L}_$r.jsonl 2>&1
    timeout -k 10 200 python3 -u bench.py --preset r18vd --precision bf16 --batch 256 --steps 10 --warmup 3 --no-cpu-baseline --latency-iters 0 --no-input-supply --no-events > $OUT/bench_c3_${L}_$r.log 2>&1
    echo "$L $r $(tail -1 $OUT/bench_c3_${L}_$r.log | cut -c1-120)"
  done
done
