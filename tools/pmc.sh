#!/bin/bash
# PMC passes for one conv shape (tools/conv_bench.py) — run on the GPU box from the repo root.
# usage: tools/pmc.sh <cfg|-> <shape-index> <outdir>
set -e
CFG=$1; IDX=$2; OUT=$3
export TMPDIR=/tmp
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/p$i -o pmc -- python3 tools/conv_bench.py $CFG $IDX > $OUT/p$i.log 2>&1
done
