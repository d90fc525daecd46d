set -euo pipefail
O=gpurun_out/${SWEEP_TAG:-sw}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "mfma16 or f32x3 or bf16" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python3 -u tools/conv_bench.py --prec ${SWEEP_PREC:-f32x3,bf16} --cfgs ${SWEEP_CFGS:-12} --shapes ${SWEEP_SHAPES:-0,1,2,3,4,5,9,11} > $O/cb.jsonl 2>&1
