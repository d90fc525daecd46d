# round 3: SQ counter passes over single GEMM shapes (tools/shape_loop.py) — tools/r3_pmc_shape.sh <tag> <shape idx...>
set -euo pipefail
OUT=gpurun_out/${1:-pmcs}; shift; mkdir -p $OUT; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" $OUT/counters.txt | sort -u > $OUT/sq_counters.txt || true
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVES"
for s in "$@"; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/s${s}_p$i -o pmc -- python3 tools/shape_loop.py $s --iters 20 > $OUT/s${s}_p$i.log 2>&1
  done
done
echo pmc done
