# round 3: A/B of split-GEMM kernel variants (tools/ab_glds.py) — tools/r3_ab.sh <tag> [pairs] [shapes]
set -euo pipefail
OUT=gpurun_out/${1:-ab}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/ab_glds.py --pairs "${2:-46:146,44:144,33:133,45:145,47:147,63:163}" ${3:+--shapes $3} --out $OUT/ab.jsonl > $OUT/ab.log 2>&1
cut -c1-220 $OUT/ab.log
