# same-box A/B of the C2 headline over this round's changes: v0 (round-5 tree), v1 (+ Winograd short-batch rule
# limited to 20000 rows), v2 (+ the three r5 interleaved re-tune entries reverted), v3 (+ element-wise split),
# and the round-4 tree
set -o pipefail
O=gpurun_out/r5u; mkdir -p $O && export TMPDIR=/tmp
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-iters 0 --no-events"
val() { python3 -c "import json;print(json.loads(open('$1').read().strip().splitlines()[-1])['value'])"; }
for i in 1 2; do
  for v in v0 v1 v2 v3; do
    SPOTTER_HIP_LIB=$PWD/spotter_amd/_ab/$v.so timeout -k 10 300 python3 -u $B > $O/${v}_$i.json 2> $O/${v}_$i.err || { tail -5 $O/${v}_$i.err; exit 1; }
  done
  (cd _r4tree && timeout -k 10 300 python3 -u $B) > $O/r4_$i.json 2> $O/r4_$i.err || { tail -5 $O/r4_$i.err; exit 1; }
  echo $i v0 $(val $O/v0_$i.json) v1 $(val $O/v1_$i.json) v2 $(val $O/v2_$i.json) v3 $(val $O/v3_$i.json) r4 $(val $O/r4_$i.json)
done
