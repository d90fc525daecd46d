# round 3: slab epilogue without a residual (cfg + 100) A/B on the non-residual split GEMMs
set -euo pipefail
OUT=gpurun_out/${1:-rd2}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/ab_glds.py --pairs "46:146,45:145,47:147,14:114,12:112,63:163,41:141,64:164" --shapes 1,2,3,4 --out $OUT/ab.jsonl > $OUT/ab.log 2>&1
grep -v '"check"' $OUT/ab.log | cut -c1-220
