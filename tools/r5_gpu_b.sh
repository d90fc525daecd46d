set -o pipefail
mkdir -p gpurun_out/r5b && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 200 --timeout-method thread -k "224_row or (fp32_accurate and (66 or 67 or 68)) or (bf16_matches and (66 or 67 or 68))" > gpurun_out/r5b/tests.log 2>&1
tail -3 gpurun_out/r5b/tests.log
timeout -k 10 600 python3 -u tools/tune_conv.py profiles/r5/x3/detail_51200_rows.json --steps 5 --modes x3 --min-ms 0.0 --reps 20 --cfgs "-,33,263,247,246,63,41,66,67,68,166,266,167,267,168,268" --out gpurun_out/r5b/tune_224.json > gpurun_out/r5b/tune.log 2>&1 || echo tune_failed
tail -2 gpurun_out/r5b/tune.log
timeout -k 10 300 python3 -u tools/detect_path.py --iters 100 > gpurun_out/r5b/detect_gpu.json 2>&1 || echo detect_failed
tail -1 gpurun_out/r5b/detect_gpu.json | cut -c1-600
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --latency-iters 0 --detail gpurun_out/r5b/detail_c2.json > gpurun_out/r5b/bench_c2.json 2> gpurun_out/r5b/bench_c2.err || echo bench_failed
tail -1 gpurun_out/r5b/bench_c2.json | cut -c1-400
