#!/bin/bash
# Round-4 (GPU box, repo root): C5 (x3) and C3 / C2-bf16 (bf16 rows) shapes re-tuned with each launch's own
# epilogue and the direct-store tile forms.
set -e
O=gpurun_out/w8
mkdir -p $O
B="python3 -u bench.py --no-cpu-baseline --latency-iters 0 --steps 5 --warmup 2"
CX="-,12,14,33,41,44,45,46,47,63,64,212,214,241,245,246,247,263,264"
CB="-,12,13,14,16,33,41,42,44,45,46,47,51,63,64,52,53,54,55,56"
timeout -k 10 300 $B --size 1280 --batch 8 --detail $O/detail_c5.json > $O/bench_c5.log 2>&1
timeout -k 10 900 python -u tools/tune_conv.py $O/detail_c5.json --steps 5 --modes x3 --min-ms 0.1 --cfgs=$CX --out $O/tune_c5_x3.json > $O/tune_c5.log 2>&1
timeout -k 10 300 $B --preset r18vd --precision bf16 --batch 256 --detail $O/detail_c3.json > $O/bench_c3.log 2>&1
timeout -k 10 900 python -u tools/tune_conv.py $O/detail_c3.json --steps 5 --modes bf16 --min-ms 0.05 --cfgs=$CB --out $O/tune_c3.json > $O/tune_c3.log 2>&1
timeout -k 10 300 $B --precision bf16 --detail $O/detail_c2bf16.json > $O/bench_c2bf16.log 2>&1
timeout -k 10 900 python -u tools/tune_conv.py $O/detail_c2bf16.json --steps 5 --modes bf16 --min-ms 0.05 --cfgs=$CB --out $O/tune_c2bf16.json > $O/tune_c2bf16.log 2>&1
