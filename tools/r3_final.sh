# round 3 final measurement pass on one MI355X: GPU tests, the default bench line (CPU baseline + latency),
# rocprof + PMC of the same bench, the config lines (C3, C2-bf16, C5), the bf16 delta, smoke.
set -euo pipefail
OUT=gpurun_out/${1:-r3f}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -1 $OUT/gpu_tests.log
if [ -d _ab_old ]; then  # same-box whole-bench A/B against the round-start tree
  ARGS="--steps 10 --warmup 3 --no-cpu-baseline --latency-iters 0"
  for i in 1 2; do
    (cd _ab_old && timeout -k 10 240 python3 -u bench.py $ARGS) > $OUT/ab_old_$i.log 2>&1
    timeout -k 10 240 python3 -u bench.py $ARGS > $OUT/ab_new_$i.log 2>&1
    echo "A/B $i old $(tail -1 $OUT/ab_old_$i.log | cut -c100-125) new $(tail -1 $OUT/ab_new_$i.log | cut -c100-125)"
  done
fi
timeout -k 10 420 python3 -u bench.py > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 > $OUT/prof.log 2>&1
python3 tools/stats_classes.py "$(find $OUT/prof -name '*kernel_stats.csv' | head -1)" --csv-out $OUT/kernel_stats.csv > $OUT/kernel_classes.json
bash tools/pmc_bench.sh $OUT/pmc > $OUT/pmc.log 2>&1
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --latency-iters 0 --detail $OUT/detail_c2.json > $OUT/bench_c2_detail.log 2>&1
tail -1 $OUT/bench_c2_detail.log | cut -c1-120
timeout -k 10 300 python3 -u bench.py --preset r18vd --batch 256 --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 --detail $OUT/detail_c3.json > $OUT/bench_c3.log 2>&1
tail -1 $OUT/bench_c3.log | cut -c1-120
timeout -k 10 300 python3 -u bench.py --precision bf16 --steps 10 --no-cpu-baseline --latency-iters 0 --detail $OUT/detail_c2bf16.json > $OUT/bench_c2bf16.log 2>&1
tail -1 $OUT/bench_c2bf16.log | cut -c1-120
timeout -k 10 300 python3 -u bench.py --size 1280 --batch 8 --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 > $OUT/bench_c5.log 2>&1
tail -1 $OUT/bench_c5.log | cut -c1-120
bash tools/pmc_bench.sh $OUT/pmc_c3 --preset r18vd --batch 256 --precision bf16 > $OUT/pmc_c3.log 2>&1
bash tools/pmc_bench.sh $OUT/pmc_c2bf16 --precision bf16 > $OUT/pmc_c2bf16.log 2>&1
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
timeout -k 10 300 python3 -u tools/bf16_delta.py bf16 --reps 8 --out $OUT/delta_bf16.json > $OUT/delta.log 2>&1
tail -1 $OUT/delta.log | cut -c1-300
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
echo final done
