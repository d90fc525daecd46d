# round 3: bf16-row slab epilogue (cfg + 100 → variant 3) A/B on the bf16 variant's residual / plain GEMMs
set -euo pipefail
OUT=gpurun_out/${1:-rd3}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/ab_glds.py --planes 1 --bf16-rows --pairs "46:146,45:145,12:112,41:141,14:114,51:151,33:133" --shapes 0,1,9,10 --out $OUT/ab.jsonl > $OUT/ab.log 2>&1
grep -v '"check"' $OUT/ab.log | cut -c1-220
