#!/bin/bash
# Round-4 (GPU box, repo root): Winograd tests on the new tiles, the C2 x3 re-tune with each launch's own
# epilogue, and a same-box A/B of the round-start tree (_abtree/r4start, git archive 4ce41ed) and this tree.
set -e
O=gpurun_out/w6
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "winograd or direct_store" > $O/t.log 2>&1
B="python3 -u bench.py --no-cpu-baseline --latency-iters 0"
for i in 1 2; do
  (cd _abtree/r4start && timeout -k 10 300 $B > ../../$O/ab_old_$i.log 2>&1)
  timeout -k 10 300 $B > $O/ab_new_$i.log 2>&1
done
timeout -k 10 300 $B --steps 5 --warmup 2 --detail $O/detail_c2.json > $O/bench_c2_detail.log 2>&1
timeout -k 10 900 python -u tools/tune_conv.py $O/detail_c2.json --steps 5 --modes x3 --min-ms 0.1 \
  --cfgs=-,12,14,33,41,44,45,46,47,63,64,212,214,241,245,246,247,263,264 --out $O/tune_c2_x3.json > $O/tune_c2_x3.log 2>&1
