# same-box A/B of the bf16 lines (C3, C2-bf16) and C5: this tree against the round-4 tree
set -o pipefail
O=gpurun_out/r5w; mkdir -p $O && export TMPDIR=/tmp
B="bench.py --steps 10 --warmup 3 --no-cpu-baseline --latency-iters 0 --no-events"
val() { python3 -c "import json;print(json.loads(open('$1').read().strip().splitlines()[-1])['value'])"; }
for i in 1 2; do
  for cfg in "c3:--preset r18vd --precision bf16 --batch 256" "c2bf16:--precision bf16" "c5:--size 1280 --batch 8"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 300 python3 -u $B $args > $O/${name}_cur_$i.json 2> $O/${name}_cur_$i.err || { tail -5 $O/${name}_cur_$i.err; exit 1; }
    (cd _r4tree && timeout -k 10 300 python3 -u $B $args) > $O/${name}_r4_$i.json 2> $O/${name}_r4_$i.err || { tail -5 $O/${name}_r4_$i.err; exit 1; }
    echo $i $name cur $(val $O/${name}_cur_$i.json) r4 $(val $O/${name}_r4_$i.json)
  done
done
