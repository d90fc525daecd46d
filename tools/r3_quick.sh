set -euo pipefail
OUT=gpurun_out/r3a; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 420 python3 -u bench.py --no-cpu-baseline --latency-iters 0 --detail $OUT/detail.json > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-400
