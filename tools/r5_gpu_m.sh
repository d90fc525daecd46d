# F(4x4) Winograd from Cin 64: bs1 A/B, C2 A/B (alternating), Winograd parity tests
set -o pipefail
O=gpurun_out/r5m; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "winograd" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python3 -u tools/bs1_ab.py --reps 100 --rounds 3 --out $O/bs1_ab.json > $O/bs1_ab.log 2>&1 || { tail -20 $O/bs1_ab.log; exit 1; }
grep variant $O/bs1_ab.log | cut -c1-250
B="python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-iters 0"
for i in 1 2; do
  timeout -k 10 300 $B > $O/c2_new_$i.json 2> $O/c2_new_$i.err || { tail -5 $O/c2_new_$i.err; exit 1; }
  tail -1 $O/c2_new_$i.json | cut -c1-120
  timeout -k 10 300 $B --wino43-min-cin 128 > $O/c2_old_$i.json 2> $O/c2_old_$i.err || { tail -5 $O/c2_old_$i.err; exit 1; }
  tail -1 $O/c2_old_$i.json | cut -c1-120
done
