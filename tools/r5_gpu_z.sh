# the staggered / persistent split kernels (cfg 70-75) against the table's tiles on the large C2 shapes
set -o pipefail
O=gpurun_out/r5z; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/retune_interleaved.py profiles/r5/x3/conv_detail_c2_r5c.json --steps 10 --rounds 3 --min-ms 0.4 --modes x3 --cands=-,70,71,72,73,74,75,246,247,245,33,63 --out $O/retune_x3sp.json > $O/retune.log 2>&1 || { tail -5 $O/retune.log; exit 1; }
tail -1 $O/retune.log
