# round-5 GPU pass: the 224-row tiles (tests + tune on the 51200-row shapes), the whole-request latency with the
# draw memo, the C2 per-shape detail, and the bs1 per-shape detail + cross-mode tune (x3 vs fp32 MFMA)
set -o pipefail
O=gpurun_out/r5c; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 200 --timeout-method thread -k "224_row or (fp32_accurate and (66 or 67 or 68)) or (bf16_matches and (66 or 67 or 68))" > $O/tests.log 2>&1
tail -3 $O/tests.log
timeout -k 10 600 python3 -u tools/tune_conv.py profiles/r5/x3/detail_51200_rows.json --steps 5 --modes x3 --min-ms 0.0 --reps 20 --cfgs "-,33,263,247,246,63,41,66,67,68,166,266,167,267,168,268" --out $O/tune_224.json > $O/tune.log 2>&1 || echo tune_failed
tail -1 $O/tune.log
timeout -k 10 300 python3 -u tools/detect_path.py --iters 100 > $O/detect_gpu.json 2>&1 || echo detect_failed
tail -1 $O/detect_gpu.json | cut -c1-700
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --latency-iters 0 --detail $O/detail_c2.json > $O/bench_c2.json 2> $O/bench_c2.err || echo bench_failed
tail -1 $O/bench_c2.json | cut -c1-300
timeout -k 10 300 python3 -u bench.py --batch 1 --steps 50 --warmup 5 --no-cpu-baseline --latency-iters 0 --detail $O/detail_bs1.json > $O/bench_bs1.json 2> $O/bench_bs1.err || echo bs1_failed
tail -1 $O/bench_bs1.json | cut -c1-300
timeout -k 10 900 python3 -u tools/tune_conv.py $O/detail_bs1.json --steps 50 --modes x3,f32 --cross --min-ms 0.004 --reps 30 --out $O/tune_bs1_cross.json > $O/tune_bs1.log 2>&1 || echo tune_bs1_failed
tail -1 $O/tune_bs1.log
