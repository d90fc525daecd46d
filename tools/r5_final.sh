#!/bin/bash
# Round-5 measurement pass (GPU box, repo root), in two calls (each under gpurun's 20-minute limit):
#   tools/r5_final.sh a <tag>   GPU suite, smoke, the driver's default line (PMC traffic first so the line carries
#                               it, CPU baseline + latency legs) and its rocprof summary
#   tools/r5_final.sh b <tag>   the config lines (C3, C2-bf16, C5 same-size and mixed stream, each with its own
#                               PMC traffic), a bs1 forward trace and the whole-request /detect path
set -euo pipefail
PART=$1
OUT=gpurun_out/${2:-r5final}; mkdir -p $OUT; export TMPDIR=/tmp
if [ "$PART" = a ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  tail -1 $OUT/gpu_tests.log
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  tail -1 $OUT/smoke.log
  bash tools/pmc_bench.sh $OUT/pmc_c2 > $OUT/pmc_c2.log 2>&1
  timeout -k 10 600 python3 -u bench.py > $OUT/bench.log 2>&1
  tail -1 $OUT/bench.log | cut -c1-200
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 > $OUT/prof.log 2>&1
  python3 tools/stats_classes.py "$(find $OUT/prof -name '*kernel_stats.csv' | head -1)" --csv-out $OUT/kernel_stats.csv > $OUT/kernel_classes.json
  echo r5_final a done
else
  B="python3 -u bench.py --no-cpu-baseline --latency-iters 0"
  for cfg in "c3:--preset r18vd --precision bf16 --batch 256" "c2bf16:--precision bf16" "c5:--size 1280 --batch 8" \
             "c5mixed:--size 1280 --batch 8 --stream mixed"; do
    name=${cfg%%:*}; args=${cfg#*:}
    bash tools/pmc_bench.sh $OUT/pmc_$name $args > $OUT/pmc_$name.log 2>&1
    timeout -k 10 300 $B $args > $OUT/bench_$name.log 2>&1
    tail -1 $OUT/bench_$name.log | cut -c1-160
  done
  cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bs1 -o bs1 -- python3 tools/latency.py --iters 40 > $OUT/latency_bs1.log 2>&1
  timeout -k 10 300 python3 -u tools/detect_path.py --iters 100 > $OUT/detect_path_gpu.json 2> $OUT/detect_path.log
  cut -c1-300 $OUT/detect_path_gpu.json
  echo r5_final b done
fi
