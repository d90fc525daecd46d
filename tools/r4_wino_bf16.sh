#!/bin/bash
# Round-4 probe (GPU box, repo root): Winograd transform variants + bf16-row GEMM tiles and PMC stall counters.
set -e
O=gpurun_out/w1
mkdir -p $O
true
true
timeout -k 10 300 python -u tools/conv_bench.py --prec bf16rows --shapes 1,28,30,9 \
  --cfgs=-,12,13,14,16,33,41,42,44,45,46,47,51,63,64 > $O/bf16_tiles.log 2>&1
timeout -k 10 600 tools/pmc.sh $O/pmc_bf16 --prec bf16rows --shapes 1,28 > $O/pmc_bf16.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/ab_wino.py --rounds 1 --reps 5 --out /tmp/x.json > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
cd $GRAFT_REPO_ROOT
timeout -k 10 600 tools/pmc.sh $O/pmc_x3 --prec f32x3 --shapes 3 > $O/pmc_x3.log 2>&1
