set -euo pipefail
OUT=gpurun_out/r3g; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --latency-iters 0 > $OUT/bench_c2.log 2>&1
tail -1 $OUT/bench_c2.log | cut -c1-160
for p in bf16 bf16-all; do
  timeout -k 10 300 python3 -u bench.py --precision $p --steps 10 --no-cpu-baseline --latency-iters 0 > $OUT/bench_c2_$p.log 2>&1
  tail -1 $OUT/bench_c2_$p.log | cut -c1-160
  timeout -k 10 300 python3 -u bench.py --preset r18vd --batch 256 --precision $p --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 > $OUT/bench_c3_$p.log 2>&1
  tail -1 $OUT/bench_c3_$p.log | cut -c1-160
  timeout -k 10 300 python3 -u tools/bf16_delta.py $p --reps 8 --out $OUT/delta_$p.json > $OUT/delta_$p.log 2>&1
  tail -1 $OUT/delta_$p.log | cut -c1-900
done
