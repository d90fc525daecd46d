#!/bin/bash
# Round 4: the C5 mixed-resolution stream line (PMC traffic first, so the bench line carries it) and a
# bs1 forward rocprof trace — run on the GPU box from the repo root:  tools/r4_c5_bs1.sh <tag>
set -euo pipefail
OUT=gpurun_out/${1:-r4}; mkdir -p $OUT; export TMPDIR=/tmp
C5="--size 1280 --batch 8 --stream mixed"
bash tools/pmc_bench.sh $OUT/pmc_c5 $C5 > $OUT/pmc_c5.log 2>&1
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
timeout -k 10 300 python3 -u bench.py $C5 --steps 6 --warmup 3 --no-cpu-baseline --latency-iters 0 \
  --detail $OUT/detail_c5.json > $OUT/bench_c5_mixed.log 2>&1
tail -1 $OUT/bench_c5_mixed.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o c5 \
  -- python3 bench.py $C5 --steps 6 --warmup 3 --no-cpu-baseline --latency-iters 0 --no-events > $OUT/prof_c5.log 2>&1
python3 tools/stats_classes.py "$(find $OUT/prof_c5 -name '*kernel_stats.csv' | head -1)" \
  --csv-out $OUT/kernel_stats_c5.csv > $OUT/kernel_classes_c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bs1 -o bs1 \
  -- python3 tools/latency.py --iters 40 > $OUT/latency_bs1.log 2>&1
tail -1 $OUT/latency_bs1.log | cut -c1-300
echo r4_c5_bs1 done
