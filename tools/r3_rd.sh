# round 3: residual-DMA epilogue (cfg + 100) A/B on the residual GEMMs
set -euo pipefail
OUT=gpurun_out/${1:-rd}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/ab_glds.py --pairs "46:146,45:145,47:147,14:114,33:133,44:144,12:112,63:163" --shapes 0,9,10,11 --out $OUT/ab.jsonl > $OUT/ab.log 2>&1
grep -v '"check"' $OUT/ab.log | cut -c1-220
timeout -k 10 300 python3 -u tools/ab_stem_c32.py --out $OUT/ab_stem.jsonl > $OUT/ab_stem.log 2>&1
cat $OUT/ab_stem.log | grep shape
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "c32" > $OUT/tests.log 2>&1
tail -1 $OUT/tests.log
