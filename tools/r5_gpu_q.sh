# Winograd transforms on buffer addressing: parity tests, then the transform rates against the previous library
set -o pipefail
O=gpurun_out/r5q; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "winograd" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
  timeout -k 10 200 python3 -u tools/microbench/wino_tf.py --reps 30 --out $O/new_$i.json > $O/new_$i.log 2>&1 || { tail -5 $O/new_$i.log; exit 1; }
  tail -1 $O/new_$i.log
  SPOTTER_HIP_LIB=$PWD/spotter_amd/_ab/libspotter_hip_base.so timeout -k 10 200 python3 -u tools/microbench/wino_tf.py --reps 30 --out $O/base_$i.json > $O/base_$i.log 2>&1 || { tail -5 $O/base_$i.log; exit 1; }
  tail -1 $O/base_$i.log
done
