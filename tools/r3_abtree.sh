# round 3: GPU tests, then a same-box A/B of the whole C2 bench — the round-start tree (_ab_old/, commit
# 8a1a6f3) vs this tree, alternating; then C3 / C2-bf16 lines
set -euo pipefail
OUT=gpurun_out/${1:-abtree}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -1 $OUT/gpu_tests.log
ARGS="--steps 10 --warmup 3 --no-cpu-baseline --latency-iters 0"
for i in 1 2; do
  (cd _ab_old && timeout -k 10 240 python3 -u bench.py $ARGS) > $OUT/old_$i.log 2>&1
  echo "old $i $(tail -1 $OUT/old_$i.log | cut -c100-140)"
  timeout -k 10 240 python3 -u bench.py $ARGS > $OUT/new_$i.log 2>&1
  echo "new $i $(tail -1 $OUT/new_$i.log | cut -c100-140)"
done
timeout -k 10 300 python3 -u bench.py --preset r18vd --batch 256 --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 > $OUT/bench_c3.log 2>&1
tail -1 $OUT/bench_c3.log | cut -c1-120
timeout -k 10 300 python3 -u bench.py --precision bf16 --steps 10 --no-cpu-baseline --latency-iters 0 > $OUT/bench_c2bf16.log 2>&1
tail -1 $OUT/bench_c2bf16.log | cut -c1-120
