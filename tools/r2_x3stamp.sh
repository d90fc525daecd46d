#!/bin/bash
# x3s iteration: stamps (diagnostic build), conv tests, sweep     tools/r2_x3stamp.sh <tag> <cfgs>
set -euo pipefail
OUT=gpurun_out/${1:-x3st}
mkdir -p "$OUT"
SPOTTER_HIP_LIB=spotter_amd/_diag/libspotter_stamp.so timeout -k 10 120 python3 tools/microbench/x3s_stamps.py --cfg 70 --shape 204800,768,768,1 > "$OUT/stamps.log" 2>&1
grep wave "$OUT/stamps.log" | grep -v median | head -8
bash tools/r2_x3.sh "$1" "$2" ""
python3 tools/sweep_table.py "$OUT/sweep.jsonl"
