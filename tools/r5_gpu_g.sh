# per-shape detail of the bf16 variant: C2-bf16 (C4's per-replica workload) and C3
set -o pipefail
O=gpurun_out/r5g; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --precision bf16 --steps 10 --warmup 3 --no-cpu-baseline --latency-iters 0 --detail $O/detail_c2bf16.json > $O/bench_c2bf16.json 2> $O/c2bf16.err || echo c2bf16_failed
tail -1 $O/bench_c2bf16.json | cut -c1-200
timeout -k 10 500 python3 -u bench.py --preset r18vd --batch 256 --precision bf16 --steps 6 --warmup 2 --no-cpu-baseline --latency-iters 0 --detail $O/detail_c3.json > $O/bench_c3.json 2> $O/c3.err || echo c3_failed
tail -1 $O/bench_c3.json | cut -c1-200
