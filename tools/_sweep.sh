set -euo pipefail
mkdir -p gpurun_out/sw1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "mfma16 or f32x3 or bf16" --timeout 120 --timeout-method thread > gpurun_out/sw1/tests.log 2>&1
tail -2 gpurun_out/sw1/tests.log
timeout -k 10 400 python3 -u tools/conv_bench.py --prec f32x3 --cfgs 12,17,18,19,20 --shapes 0,1,2,3,4,5,9,11 > gpurun_out/sw1/cb.jsonl 2>&1
timeout -k 10 300 python3 -u tools/conv_bench.py --prec fp32,f32x3 --cfgs - --shapes 6,7,8,10,12,13,14,15,16 > gpurun_out/sw1/cb_small.jsonl 2>&1
