set -o pipefail
O=gpurun_out/ax2; mkdir -p $O
for t in old new old new; do
  if [ $t = old ]; then L=$PWD/_ab/lib_old.so; else L=$PWD/spotter_amd/libspotter_hip.so; fi
  SPOTTER_HIP_LIB=$L timeout -k 10 180 python -u tools/microbench/attn_ab.py --tag $t > $O/xcd_$t.$RANDOM.jsonl || exit 1
done
for t in old new old new; do
  if [ $t = old ]; then L=$PWD/_ab/lib_old.so; else L=$PWD/spotter_amd/libspotter_hip.so; fi
  SPOTTER_HIP_LIB=$L timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --latency-iters 0 --preset r18vd --precision bf16 --batch 256 > $O/c3_$t.$RANDOM.log 2>&1 || exit 1
done
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
echo done
