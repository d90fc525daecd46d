#!/bin/bash
# Round-6 GPU passes (GPU box, repo root):
#   tools/r6_gpu.sh serve <tag>   GPU suite, the k-replicas-per-GPU whole-request sweep (fp32, bf16), the bench's
#                                 default line with its input-supply leg, the MSDA gather ceiling, x3 stage-3 PMC
set -euo pipefail
PART=$1
OUT=gpurun_out/${2:-r6}; mkdir -p $OUT; export TMPDIR=/tmp
if [ "$PART" = serve ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  tail -1 $OUT/gpu_tests.log
  timeout -k 10 600 python3 -u tools/served_sweep.py --k 1 2 4 --precision fp32 bf16 --seconds 8 --out $OUT/served > $OUT/served.log 2>&1
  cat $OUT/served.log | cut -c1-240
  timeout -k 10 300 python3 -u tools/microbench/gather_ceiling.py --out $OUT/gather_ceiling.json > $OUT/gather.log 2>&1
  tail -1 $OUT/gather.log | cut -c1-400
  timeout -k 10 600 python3 -u bench.py > $OUT/bench.log 2>&1
  tail -1 $OUT/bench.log | cut -c1-200
  bash tools/pmc.sh $OUT/pmc_x3 --prec f32x3 --shapes 3,4 > $OUT/pmc_x3.log 2>&1
  tail -5 $OUT/pmc_x3.log
  echo r6 serve done
fi
if [ "$PART" = bounds ]; then
  # product library: GPU suite + MSDA A/B; then the bounds-check library over the same suite; then the served sweep
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  tail -1 $OUT/gpu_tests.log
  timeout -k 10 300 python3 -u tools/microbench/msda_ab.py --out $OUT/msda_ab.json > $OUT/msda_ab.log 2>&1
  cat $OUT/msda_ab.log | grep -v amdgpu.ids | cut -c1-300
  set +e
  SPOTTER_HIP_LIB=spotter_amd/_bounds/libspotter_bounds.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_tests_bounds.log 2>&1
  rc=$?
  set -e
  tail -3 $OUT/gpu_tests_bounds.log
  # test failures (rc 1) are the report; a crash, abort or time limit ends the call here
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "bounds suite rc=$rc: stopping"; exit $rc; fi
  cp gpurun_out/bounds_report.json $OUT/bounds_report.json 2>/dev/null || true
  timeout -k 10 900 python3 -u tools/served_sweep.py --k 6 8 12 --precision bf16 fp32 --seconds 8 --out $OUT/served > $OUT/served.log 2>&1
  grep -v amdgpu.ids $OUT/served.log | cut -c1-240
  echo r6 bounds done
fi
if [ "$PART" = quick ]; then
  SPOTTER_HIP_LIB=spotter_amd/_bounds/libspotter_bounds.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -q -k "bounds_build or gather_rows" --timeout 120 --timeout-method thread > $OUT/bounds_control.log 2>&1
  tail -2 $OUT/bounds_control.log
  timeout -k 10 300 python3 -u bench.py --size 1280 --batch 8 --stream mixed --no-cpu-baseline --latency-iters 0 --no-input-supply > $OUT/bench_c5mixed.log 2>&1
  tail -1 $OUT/bench_c5mixed.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['kernel_classes']['preprocess']), json.dumps(d['kernel_classes']['msda']))"
  timeout -k 10 300 python3 -u tools/microbench/gather_ceiling.py --out $OUT/gather_ceiling.json > $OUT/gather.log 2>&1
  tail -1 $OUT/gather.log | cut -c1-600
  echo r6 quick done
fi
if [ "$PART" = pre ]; then
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -k "preprocess or mixed_resolution" --timeout 200 --timeout-method thread > $OUT/pre_tests.log 2>&1
  tail -1 $OUT/pre_tests.log
  for i in 1 2; do
    timeout -k 10 300 python3 -u bench.py --size 1280 --batch 8 --stream mixed --no-cpu-baseline --latency-iters 0 --no-input-supply > $OUT/bench_c5mixed_$i.log 2>&1
    tail -1 $OUT/bench_c5mixed_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['kernel_classes']['preprocess']))"
  done
  echo r6 pre done
fi
