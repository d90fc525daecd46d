# split-K reduce with every split's load in flight: parity tests, then the bs1 forward against the previous library
set -o pipefail
O=gpurun_out/r5y; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "split" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2 3; do
  timeout -k 10 200 python3 -u tools/latency.py --iters 200 > $O/new_$i.json 2> $O/new_$i.err || { tail -5 $O/new_$i.err; exit 1; }
  SPOTTER_HIP_LIB=$PWD/spotter_amd/_ab/base.so timeout -k 10 200 python3 -u tools/latency.py --iters 200 > $O/base_$i.json 2> $O/base_$i.err || { tail -5 $O/base_$i.err; exit 1; }
  python3 -c "import json;a=json.load(open('$O/new_$i.json'));b=json.load(open('$O/base_$i.json'));print('new',a['forward_p50_ms'],a['p50_ms'],'base',b['forward_p50_ms'],b['p50_ms'])"
done
