# interleaved tile re-tune of the C2 GEMM shapes (x3 and fp32 MFMA) with >= 0.1 ms per step
set -o pipefail
O=gpurun_out/r5e; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 1000 python3 -u tools/retune_interleaved.py profiles/r5/x3/conv_detail_c2_r5c.json --steps 10 --rounds 5 --min-ms 0.1 --out $O/retune_c2.json > $O/retune.log 2>&1 || echo retune_failed
tail -1 $O/retune.log
