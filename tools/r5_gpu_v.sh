# same-box A/B of the C2 headline: v4 (round-5 tree, counters path compiled only into the split-K instances,
# scalar split) / v3 (element-wise split, counters path in every epilogue) / the round-4 tree
set -o pipefail
O=gpurun_out/r5v; mkdir -p $O && export TMPDIR=/tmp
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-iters 0 --no-events"
val() { python3 -c "import json;print(json.loads(open('$1').read().strip().splitlines()[-1])['value'])"; }
for i in 1 2 3; do
  for v in v4 v3; do
    SPOTTER_HIP_LIB=$PWD/spotter_amd/_ab/$v.so timeout -k 10 300 python3 -u $B > $O/${v}_$i.json 2> $O/${v}_$i.err || { tail -5 $O/${v}_$i.err; exit 1; }
  done
  (cd _r4tree && timeout -k 10 300 python3 -u $B) > $O/r4_$i.json 2> $O/r4_$i.err || { tail -5 $O/r4_$i.err; exit 1; }
  echo $i v4 $(val $O/v4_$i.json) v3 $(val $O/v3_$i.json) r4 $(val $O/r4_$i.json)
done
