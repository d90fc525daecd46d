# round 3: tile choice with the slab epilogue on the C2 split-mode shapes (the table's tile vs slab-enabled tiles)
set -euo pipefail
OUT=gpurun_out/${1:-tiles}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/ab_glds.py --no-check --pairs "33:163,33:141,33:112,42:141,42:163,46:147,46:145,44:147,44:163" --shapes 0,1,2,3,4,9,10,11 --out $OUT/ab.jsonl > $OUT/ab.log 2>&1
cut -c1-200 $OUT/ab.log
