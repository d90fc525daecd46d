# 256x256 deep-stage bf16-row tiles (cfg 57-59): bit-identity, then interleaved re-tune of the long-K bf16 shapes
set -o pipefail
O=gpurun_out/r5p; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "bf16_a_rows_bit_identical or bf16_rows_in_and_out" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
C="-,41,53,55,33,52,57,58,59"
timeout -k 10 500 python3 -u tools/retune_interleaved.py profiles/r5/bf16/detail_c3.json --steps 6 --rounds 3 --min-ms 0.3 --modes bf16 --cands=$C --out $O/retune_c3.json > $O/retune_c3.log 2>&1 || { tail -5 $O/retune_c3.log; exit 1; }
tail -1 $O/retune_c3.log
timeout -k 10 400 python3 -u tools/retune_interleaved.py profiles/r5/bf16/detail_c2bf16.json --steps 10 --rounds 3 --min-ms 0.3 --modes bf16 --cands=$C --out $O/retune_c2bf16.json > $O/retune_c2bf16.log 2>&1 || { tail -5 $O/retune_c2bf16.log; exit 1; }
tail -1 $O/retune_c2bf16.log
