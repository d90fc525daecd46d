# after moving conv_x3s / conv_x3p to the diagnostic build: the GPU suite, the smoke and a short C2 line
set -o pipefail
O=gpurun_out/r5aa; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-iters 0 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-160
