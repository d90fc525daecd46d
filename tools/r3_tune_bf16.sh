# round 3: bf16 operand mode — A/B of the 64-deep stage tiles, then per-shape tuning of C2-bf16 and C3
set -euo pipefail
OUT=gpurun_out/${1:-r3bf16}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/ab_glds.py --planes 1 --pairs 45:52,12:56 --rounds 3 --reps 8 --out $OUT/ab_bk64_bf16.jsonl > $OUT/ab_bf16.log 2>&1
grep -c '"bit_identical": true' $OUT/ab_bf16.log
timeout -k 10 300 python3 -u tools/ab_glds.py --planes 3 --pairs 45:52 --rounds 3 --reps 8 --out $OUT/ab_bk64_x3.jsonl > $OUT/ab_x3.log 2>&1
grep '"shape"' $OUT/ab_bf16.log $OUT/ab_x3.log | cut -c1-220
timeout -k 10 300 python3 -u bench.py --precision bf16 --steps 10 --no-cpu-baseline --latency-iters 0 --detail $OUT/detail_c2bf16.json > $OUT/bench_c2bf16.log 2>&1
tail -1 $OUT/bench_c2bf16.log | cut -c1-200
timeout -k 10 300 python3 -u bench.py --preset r18vd --batch 256 --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --latency-iters 0 --detail $OUT/detail_c3.json > $OUT/bench_c3.log 2>&1
tail -1 $OUT/bench_c3.log | cut -c1-200
C="-,11,12,13,14,16,17,33,41,42,44,45,46,47,49,51,52,53,54,55,56,63"
timeout -k 10 900 python3 -u tools/tune_conv.py $OUT/detail_c2bf16.json --modes bf16 --min-ms 0.1 --cfgs=$C --out $OUT/tune_c2bf16.json --reps 6 > $OUT/tune_c2bf16.log 2>&1
tail -1 $OUT/tune_c2bf16.log
timeout -k 10 900 python3 -u tools/tune_conv.py $OUT/detail_c3.json --steps 5 --modes bf16 --min-ms 0.1 --cfgs=$C --out $OUT/tune_c3.json --reps 6 > $OUT/tune_c3.log 2>&1
tail -1 $OUT/tune_c3.log
