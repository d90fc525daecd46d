#!/bin/bash
# Round-4 bf16-row tile study (GPU box, repo root): new deeper-pipeline configs on the bf16 3x3s, then the
# C3 / C2-bf16 steps' own shapes re-tuned in the bf16-row form they run in.
set -e
O=gpurun_out/w2
mkdir -p $O
CF="-,12,13,14,16,33,41,42,44,45,46,47,51,63,64,52,53,54,55,56"
timeout -k 10 300 python -u tools/conv_bench.py --prec bf16rows --shapes 1,28,30,9 --cfgs=-,12,41,47,52,53,54,55,56 > $O/bf16_new_cfgs.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-iters 0 --preset r18vd --precision bf16 --batch 256 --steps 5 --warmup 2 --detail $O/detail_c3.json > $O/bench_c3.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-iters 0 --precision bf16 --steps 5 --warmup 2 --detail $O/detail_c2bf16.json > $O/bench_c2bf16.log 2>&1
timeout -k 10 600 python -u tools/tune_conv.py $O/detail_c3.json --steps 5 --modes bf16 --cfgs=$CF --out $O/tune_c3.json > $O/tune_c3.log 2>&1
timeout -k 10 600 python -u tools/tune_conv.py $O/detail_c2bf16.json --steps 5 --modes bf16 --cfgs=$CF --out $O/tune_c2bf16.json > $O/tune_c2bf16.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "winograd" > $O/t_wino.log 2>&1
timeout -k 10 300 python -u tools/ab_wino.py --out $O/ab_wino.json > $O/ab_wino.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_wino -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_wino.py --rounds 1 --reps 5 --out /tmp/x.json > $GRAFT_REPO_ROOT/$O/prof_wino.log 2>&1
cd $GRAFT_REPO_ROOT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "direct_store" > $O/t_dstore.log 2>&1
timeout -k 10 400 python -u tools/ab_glds.py --pairs 146:246,147:247,145:245,163:263,112:212,141:241 --shapes 0,9,10,11,1,4,2 --out $O/ab_dstore.jsonl > $O/ab_dstore.log 2>&1
for c in 46 47 63; do SPOTTER_HIP_LIB=spotter_amd/_diag/libspotter_stamp.so timeout -k 10 120 python -u tools/microbench/glds_stamps.py 0 --cfg $c >> $O/stamps.jsonl 2>>$O/stamps.err; done
SPOTTER_HIP_LIB=spotter_amd/_diag/libspotter_stamp.so timeout -k 10 120 python -u tools/microbench/glds_stamps.py 1 --cfg 33 >> $O/stamps.jsonl 2>>$O/stamps.err
