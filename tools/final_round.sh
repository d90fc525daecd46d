set -euo pipefail
OUT=gpurun_out/${1:-r1_final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -1 $OUT/gpu_tests.log
bash tools/pmc_bench.sh $OUT/pmc > $OUT/pmc.log 2>&1
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
timeout -k 10 420 python3 -u bench.py > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 > $OUT/prof.log 2>&1
python3 tools/stats_classes.py "$(find $OUT/prof -name '*kernel_stats.csv' | head -1)" --csv-out $OUT/kernel_stats.csv > $OUT/kernel_classes.json
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
echo final done
