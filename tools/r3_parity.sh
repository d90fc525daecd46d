# round 3: golden parity (with margins) + the bf16 delta on the current tree
set -euo pipefail
OUT=gpurun_out/${1:-r3p}; mkdir -p $OUT; export TMPDIR=/tmp
export SPOTTER_MARGINS_OUT=$OUT/parity_margins.json
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_model.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_model.log 2>&1 || true
tail -3 $OUT/gpu_model.log
timeout -k 10 400 python3 -u tools/bf16_delta.py bf16 --reps 8 --out $OUT/bf16_delta.json > $OUT/bf16.log 2>&1
tail -1 $OUT/bf16.log | cut -c1-600
