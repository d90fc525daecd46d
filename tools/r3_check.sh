# round 3: GPU tests + the config lines + bf16 delta on the current tree (no profiler passes)
set -euo pipefail
OUT=gpurun_out/${1:-chk}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --latency-iters 0 --detail $OUT/detail_c2.json > $OUT/bench_c2.log 2>&1
tail -1 $OUT/bench_c2.log | cut -c1-120
timeout -k 10 300 python3 -u bench.py --preset r18vd --batch 256 --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 --detail $OUT/detail_c3.json > $OUT/bench_c3.log 2>&1
tail -1 $OUT/bench_c3.log | cut -c1-120
timeout -k 10 300 python3 -u bench.py --precision bf16 --steps 10 --no-cpu-baseline --latency-iters 0 --detail $OUT/detail_c2bf16.json > $OUT/bench_c2bf16.log 2>&1
tail -1 $OUT/bench_c2bf16.log | cut -c1-120
timeout -k 10 300 python3 -u tools/bf16_delta.py bf16 --reps 8 --out $OUT/delta_bf16.json > $OUT/delta.log 2>&1
tail -1 $OUT/delta.log | cut -c1-400
echo check done
