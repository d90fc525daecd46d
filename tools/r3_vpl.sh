# round 3: Winograd V as split bf16 planes / bf16 A planes — bit-identity tests, then the A/B
set -euo pipefail
OUT=gpurun_out/${1:-vpl}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "v_planes or a_planes or winograd" > $OUT/tests.log 2>&1
tail -2 $OUT/tests.log
timeout -k 10 400 python3 -u tools/ab_glds.py --no-check --pairs "46:46v,44:44v,47:47v,14:14v" --shapes 5,6,7,8 --out $OUT/ab.jsonl > $OUT/ab.log 2>&1
cut -c1-200 $OUT/ab.log
