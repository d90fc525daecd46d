#!/bin/bash
# PMC passes over tools/conv_bench.py — run on the GPU box from the repo root:
#   tools/pmc.sh <outdir> <conv_bench args...>      e.g. tools/pmc.sh gpurun_out/pmc --prec f32x3 --cfgs=1 --shapes 1
# One rocprofv3 run per counter pass (each within gfx950's per-block limits), --kernel-trace only,
# then tools/pmc_summary.py prints per-kernel means.
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/p$i" -o pmc \
    -- python3 tools/conv_bench.py "$@" > "$OUT/p$i.log" 2>&1
done
python3 tools/pmc_summary.py "$OUT"
