set -euo pipefail
mkdir -p gpurun_out/abl
for A in 0 1 2 3; do
  if [ $A = 0 ]; then L=spotter_amd/libspotter_hip.so; else L=spotter_amd/_ablate/lib_$A.so; fi
  SPOTTER_HIP_LIB=$L timeout -k 10 200 python3 -u tools/conv_bench.py --prec f32x3,bf16 --cfgs 12,11 --shapes 0,1,3 > gpurun_out/abl/a$A.jsonl 2>&1
done
