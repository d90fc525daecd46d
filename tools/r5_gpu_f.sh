# same-box A/B of the packed-pair split (product library) against the scalar-subtraction split
# (spotter_amd/_diag/libspotter_oldsplit.so, -DSP_SPLIT_PK2=0): output checksums, then alternating C2 benches
set -o pipefail
O=gpurun_out/r5f; mkdir -p $O && export TMPDIR=/tmp
OLD=spotter_amd/_diag/libspotter_oldsplit.so
SPOTTER_HIP_LIB=$OLD timeout -k 10 300 python3 -u tools/ab_lib_checksums.py > $O/ck_old.txt 2>&1 || echo ck_old_failed
timeout -k 10 300 python3 -u tools/ab_lib_checksums.py > $O/ck_new.txt 2>&1 || echo ck_new_failed
tail -1 $O/ck_old.txt; tail -1 $O/ck_new.txt
for i in 1 2 3; do
  SPOTTER_HIP_LIB=$OLD timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --latency-iters 0 > $O/old_$i.json 2>/dev/null || echo old_failed
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --latency-iters 0 > $O/new_$i.json 2>/dev/null || echo new_failed
  python3 -c "import json,sys; [print(f, json.loads(open(f).read().strip().split(chr(10))[-1])['value'], json.loads(open(f).read().strip().split(chr(10))[-1])['roofline']['frac']) for f in sys.argv[1:]]" $O/old_$i.json $O/new_$i.json
done
