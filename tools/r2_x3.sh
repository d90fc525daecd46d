#!/bin/bash
# x3 kernel iteration on the GPU box: correctness of every tile config, the per-shape sweep,
# and one SQ/GRBM counter pass per config on the dominant shape.   tools/r2_x3.sh <tag> <cfgs> [pmc cfgs]
set -euo pipefail
OUT=gpurun_out/${1:-x3}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q -k "conv2d" --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -1 "$OUT/tests.log"
timeout -k 10 400 python3 -u tools/conv_bench.py --prec f32x3 --cfgs="$2" --shapes 0,1,2,3,4,5,6 --reps 10 > "$OUT/sweep.jsonl" 2>&1
for c in ${3:-}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d "$OUT/pmc_$c" -o p -- python3 tools/conv_bench.py --prec f32x3 --cfgs=$c --shapes 0,1 --reps 3 > "$OUT/pmc_$c.log" 2>&1
done
echo x3 done
