# A/B of LDS-DMA GEMM tile configurations / epilogue variants on the GPU box (tools/ab_glds.py, interleaved,
# bit-identity checked), e.g. tools/gpu_ab.sh rd --pairs "46:146,45:145" --shapes 0,9,10,11 [--planes 1 --bf16-rows]
set -euo pipefail
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/ab_glds.py "$@" --out "$OUT/ab.jsonl" > "$OUT/ab.log" 2>&1
grep -v '"check"' "$OUT/ab.log" | cut -c1-220
