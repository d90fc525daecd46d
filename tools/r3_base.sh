set -euo pipefail
OUT=gpurun_out/${1:-r3a}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --latency-iters 0 --detail $OUT/detail_c2.json > $OUT/bench_c2.log 2>&1
tail -1 $OUT/bench_c2.log | cut -c1-200
