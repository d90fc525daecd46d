# round 3: bf16 activation storage — kernel + model tests, then C3 / C2-bf16 benches (bf16 maps vs fp32 maps), delta
set -euo pipefail
OUT=gpurun_out/${1:-bf}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "bf16 or a_planes or v_planes" > $OUT/tests.log 2>&1
tail -2 $OUT/tests.log
for M in "" "--fp32-maps"; do
  timeout -k 10 300 python3 -u bench.py --preset r18vd --batch 256 --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 $M > $OUT/bench_c3$M.log 2>&1
  tail -1 $OUT/bench_c3$M.log | cut -c1-150
  timeout -k 10 300 python3 -u bench.py --precision bf16 --steps 10 --no-cpu-baseline --latency-iters 0 $M > $OUT/bench_c2bf16$M.log 2>&1
  tail -1 $OUT/bench_c2bf16$M.log | cut -c1-150
done
timeout -k 10 300 python3 -u tools/bf16_delta.py bf16 --reps 8 --out $OUT/delta_bf16.json > $OUT/delta.log 2>&1
tail -1 $OUT/delta.log | cut -c1-900
