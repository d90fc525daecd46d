# bs1: post-LayerNorms fused into the GEMM epilogue (diagnostic build's fused-LN tiles) against the unfused form
set -o pipefail
O=gpurun_out/r5x; mkdir -p $O && export TMPDIR=/tmp
SPOTTER_HIP_LIB=$PWD/spotter_amd/_ab/diag_ln.so timeout -k 10 300 python3 -u tools/bs1_ab.py --reps 100 --rounds 3 --variants plain:-1:16:8,ln:-1:16:8 --out $O/bs1_ab_ln.json > $O/bs1_ab_ln.log 2>&1 || { tail -20 $O/bs1_ab_ln.log; exit 1; }
grep variant $O/bs1_ab_ln.log | cut -c1-250
