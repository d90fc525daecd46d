# round 3: re-tune x3 tiles for the bs32 C2 shapes on the current kernels, and the F(4x4) component GEMMs
set -euo pipefail
OUT=gpurun_out/${1:-r3tune}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --latency-iters 0 --detail $OUT/detail.json > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-200
timeout -k 10 900 python3 -u tools/tune_conv.py $OUT/detail.json --modes x3 --min-ms 0.1 --out $OUT/tune_x3.json --reps 8 > $OUT/tune_x3.log 2>&1
tail -1 $OUT/tune_x3.log
timeout -k 10 600 python3 -u tools/tune_wino.py --m 4 --cfgs 11,12,14,16,17,33,41,44,45,46,47,48,49,63,64 --shapes "32,80,80,384,384;32,40,40,384,384;32,20,20,384,384;32,40,40,256,256;32,20,20,512,512;32,80,80,128,128" --out $OUT/tune_wino_f43.json --reps 8 > $OUT/tune_wino.log 2>&1
cut -c1-300 $OUT/tune_wino.log
