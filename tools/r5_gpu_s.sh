# stem conv 1 with two pixels per lane (packed FMAs): bit-identity and time against the previous library
set -o pipefail
O=gpurun_out/r5s; mkdir -p $O && export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python3 -u tools/microbench/stem_ab.py > $O/new_$i.json 2> $O/new_$i.err || { tail -5 $O/new_$i.err; exit 1; }
  SPOTTER_HIP_LIB=$PWD/spotter_amd/_ab/libspotter_hip_base.so timeout -k 10 200 python3 -u tools/microbench/stem_ab.py > $O/base_$i.json 2> $O/base_$i.err || { tail -5 $O/base_$i.err; exit 1; }
done
cat $O/new_1.json $O/base_1.json $O/new_2.json $O/base_2.json
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "stem" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
