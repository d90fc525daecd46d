# Pool / upsample A/B: the previous library (_ab/lib_old.so, copied in by hand) vs the in-tree one, alternating
# processes on one box, then the pool / upsample GPU tests. Run on the GPU box from the repo root.
set -o pipefail
O=gpurun_out/${1:-up}; mkdir -p $O
for t in old new old new; do
  if [ $t = old ]; then L=$PWD/_ab/lib_old.so; else L=$PWD/spotter_amd/libspotter_hip.so; fi
  SPOTTER_HIP_LIB=$L timeout -k 10 180 python -u tools/microbench/pool_ab.py --tag $t > $O/$t.$RANDOM.jsonl || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "pool or upsample or bf16_rows" > $O/tests.log 2>&1 || exit 1
echo done
