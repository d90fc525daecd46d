#!/bin/bash
# Round-4 check (GPU box, repo root): the whole GPU suite, the bf16 configs after the bf16-row re-tune, the
# direct-store epilogue A/B and the expand's per-workgroup stamps.
set -e
O=gpurun_out/w3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
B="python3 -u bench.py --no-cpu-baseline --latency-iters 0"
timeout -k 10 300 $B --preset r18vd --precision bf16 --batch 256 --detail $O/detail_c3.json > $O/bench_c3.log 2>&1
timeout -k 10 300 $B --precision bf16 --detail $O/detail_c2bf16.json > $O/bench_c2bf16.log 2>&1
timeout -k 10 400 python -u tools/ab_glds.py --pairs 146:246,147:247,145:245,163:263,112:212,141:241 --shapes 0,9,10,11,1,4,2 --out $O/ab_dstore.jsonl > $O/ab_dstore.log 2>&1
for c in 46 47 63; do SPOTTER_HIP_LIB=spotter_amd/_diag/libspotter_stamp.so timeout -k 10 120 python -u tools/microbench/glds_stamps.py 0 --cfg $c >> $O/stamps.jsonl 2>>$O/stamps.err; done
SPOTTER_HIP_LIB=spotter_amd/_diag/libspotter_stamp.so timeout -k 10 120 python -u tools/microbench/glds_stamps.py 1 --cfg 33 >> $O/stamps.jsonl 2>>$O/stamps.err
