#!/bin/bash
# Round-6 measurement pass (GPU box, repo root), two calls (each under gpurun's 20-minute limit):
#   tools/r6_final.sh a <tag>   GPU suite, smoke, the driver's default line (PMC traffic first so the line carries
#                               it; CPU baseline, latency and input-supply legs), its rocprof summary, then the GPU
#                               suite once more on the bounds-check library
#   tools/r6_final.sh b <tag>   the config lines (C3, C2-bf16, C5 same-size and mixed stream, each with its own PMC
#                               traffic), a bs1 forward trace, the whole-request /detect path, a C3 rocprof summary
set -euo pipefail
PART=$1
OUT=gpurun_out/${2:-r6final}; mkdir -p $OUT; export TMPDIR=/tmp
if [ "$PART" = a ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  tail -1 $OUT/gpu_tests.log
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  tail -1 $OUT/smoke.log
  bash tools/pmc_bench.sh $OUT/pmc_c2 > $OUT/pmc_c2.log 2>&1
  cp profiles/pmc_traffic.json $OUT/pmc_traffic_a.json
  timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1
  tail -1 $OUT/bench.log | cut -c1-200
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 --no-input-supply > $OUT/prof.log 2>&1
  python3 tools/stats_classes.py "$(find $OUT/prof -name '*kernel_stats.csv' | head -1)" --csv-out $OUT/kernel_stats.csv > $OUT/kernel_classes.json
  set +e
  SPOTTER_HIP_LIB=spotter_amd/_bounds/libspotter_bounds.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_bounds.log 2>&1
  rc=$?
  set -e
  tail -1 $OUT/gpu_tests_bounds.log
  cp gpurun_out/bounds_report.json $OUT/bounds_report.json 2>/dev/null || true
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "bounds suite rc=$rc"; exit $rc; fi
  echo r6_final a done
else
  B="python3 -u bench.py --no-cpu-baseline --latency-iters 0 --no-input-supply"
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
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o c3 -- python3 bench.py --preset r18vd --precision bf16 --batch 256 --steps 4 --warmup 2 --no-cpu-baseline --latency-iters 0 --no-input-supply --no-events > $OUT/prof_c3.log 2>&1
  python3 tools/stats_classes.py "$(find $OUT/prof_c3 -name '*kernel_stats.csv' | head -1)" --csv-out $OUT/kernel_stats_c3.csv > $OUT/kernel_classes_c3.json
  echo r6_final b done
fi
