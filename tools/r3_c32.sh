# round 3: direct bf16 stem 3x3 — test, then C3 / C2-bf16 benches
set -euo pipefail
OUT=gpurun_out/${1:-c32}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "c32 or bf16" > $OUT/tests.log 2>&1
tail -2 $OUT/tests.log
timeout -k 10 300 python3 -u bench.py --preset r18vd --batch 256 --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 --detail $OUT/detail_c3.json > $OUT/bench_c3.log 2>&1
tail -1 $OUT/bench_c3.log | cut -c1-150
timeout -k 10 300 python3 -u bench.py --precision bf16 --steps 10 --no-cpu-baseline --latency-iters 0 > $OUT/bench_c2bf16.log 2>&1
tail -1 $OUT/bench_c2bf16.log | cut -c1-150
