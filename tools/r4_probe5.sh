#!/bin/bash
# Round-4 (GPU box, repo root): whole GPU suite on the re-tuned tables, then a same-box A/B of the round-start
# tree and this tree (C2), and the C3 / C2-bf16 lines.
set -e
O=gpurun_out/w7
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
B="python3 -u bench.py --no-cpu-baseline --latency-iters 0"
for i in 1 2; do
  (cd _abtree/r4start && timeout -k 10 300 $B > ../../$O/ab_old_$i.log 2>&1)
  timeout -k 10 300 $B > $O/ab_new_$i.log 2>&1
done
(cd _abtree/r4start && timeout -k 10 300 $B --preset r18vd --precision bf16 --batch 256 > ../../$O/ab_old_c3.log 2>&1)
timeout -k 10 300 $B --preset r18vd --precision bf16 --batch 256 > $O/ab_new_c3.log 2>&1
(cd _abtree/r4start && timeout -k 10 300 $B --precision bf16 > ../../$O/ab_old_c2bf16.log 2>&1)
timeout -k 10 300 $B --precision bf16 > $O/ab_new_c2bf16.log 2>&1
