# transposed-roles bf16 epilogue (cfg + 300): parity tests, then interleaved re-tune of the C3 / C2-bf16 shapes
set -o pipefail
O=gpurun_out/r5h; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "transposed_roles or bf16_rows or bf16_a_rows" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 500 python3 -u tools/retune_interleaved.py profiles/r5/bf16/detail_c3.json --steps 6 --rounds 3 --min-ms 0.25 --modes bf16 --out $O/retune_c3.json > $O/retune_c3.log 2>&1 || { tail -5 $O/retune_c3.log; exit 1; }
tail -1 $O/retune_c3.log
timeout -k 10 400 python3 -u tools/retune_interleaved.py profiles/r5/bf16/detail_c2bf16.json --steps 10 --rounds 3 --min-ms 0.15 --modes bf16 --out $O/retune_c2bf16.json > $O/retune_c2bf16.log 2>&1 || { tail -5 $O/retune_c2bf16.log; exit 1; }
tail -1 $O/retune_c2bf16.log
