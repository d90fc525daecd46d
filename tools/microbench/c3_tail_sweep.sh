#!/bin/bash
# C3's decoder / encoder-head GEMM shapes over every LDS-DMA tile (tools/conv_bench.py shapes 31-38)
set -euo pipefail
OUT=${1:-gpurun_out/c3tail}; mkdir -p $OUT
CF="-,11,12,13,14,15,16,33,34,35,36,37,38,41,42,43,44,45,46,47,48,49,50,51,62,63,64,65"
timeout -k 10 300 python3 -u tools/conv_bench.py --prec bf16rows --shapes 31,37 --cfgs=$CF --reps 10 > $OUT/rows16.jsonl 2>&1
timeout -k 10 300 python3 -u tools/conv_bench.py --prec bf16 --shapes 32,33,34,35,36,38 --cfgs=$CF --reps 20 > $OUT/dec_bf16.jsonl 2>&1
