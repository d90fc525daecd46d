# round 3: per-shape conv detail + PMC HBM traffic of the bf16 configs (C3, C2-bf16) on the current tree
set -euo pipefail
OUT=gpurun_out/${1:-det}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --preset r18vd --batch 256 --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 --detail $OUT/detail_c3.json > $OUT/bench_c3.log 2>&1
tail -1 $OUT/bench_c3.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py --precision bf16 --steps 10 --no-cpu-baseline --latency-iters 0 --detail $OUT/detail_c2bf16.json > $OUT/bench_c2bf16.log 2>&1
tail -1 $OUT/bench_c2bf16.log | cut -c1-200
bash tools/pmc_bench.sh $OUT/pmc_c3 --preset r18vd --batch 256 --precision bf16 > $OUT/pmc_c3.log 2>&1
bash tools/pmc_bench.sh $OUT/pmc_c2bf16 --precision bf16 > $OUT/pmc_c2bf16.log 2>&1
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
echo detail done
