# in-launch split-K combine: parity tests, then the bs1 forward A/B against the separate reduce launch
set -o pipefail
O=gpurun_out/r5j; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "split" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 400 python3 -u tools/bs1_ab.py --reps 100 --rounds 3 --out $O/bs1_ab.json > $O/bs1_ab.log 2>&1 || { tail -20 $O/bs1_ab.log; exit 1; }
grep variant $O/bs1_ab.log | cut -c1-300
