# the 224-row tiles against the table / by-shape choice on the 51200-row C2 shapes (same box, interleaved reps)
set -o pipefail
O=gpurun_out/r5d; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python3 -u tools/tune_conv.py profiles/r5/x3/detail_51200_rows.json --steps 5 --modes x3 --min-ms 0.0 --reps 20 --cfgs=-,33,263,247,246,63,41,66,67,68,166,266,167,267,168,268 --out $O/tune_224.json > $O/tune.log 2>&1 || echo tune_failed
tail -1 $O/tune.log
