set -euo pipefail
OUT=gpurun_out/r3d; mkdir -p $OUT; export TMPDIR=/tmp
for b in 32 16 8; do
  timeout -k 10 300 python3 -u bench.py --batch $b --steps 10 --no-cpu-baseline --latency-iters 0 --no-events > $OUT/bench_bs$b.log 2>&1
  tail -1 $OUT/bench_bs$b.log | cut -c1-200
done
