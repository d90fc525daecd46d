# same-box A/B of the C2 headline: this tree against the round-4 tree (_r4tree, built from its own sources)
set -o pipefail
O=gpurun_out/r5t; mkdir -p $O && export TMPDIR=/tmp
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-iters 0 --no-events"
for i in 1 2 3; do
  timeout -k 10 300 python3 -u $B > $O/cur_$i.json 2> $O/cur_$i.err || { tail -5 $O/cur_$i.err; exit 1; }
  (cd _r4tree && timeout -k 10 300 python3 -u $B) > $O/r4_$i.json 2> $O/r4_$i.err || { tail -5 $O/r4_$i.err; exit 1; }
  echo $i cur $(python3 -c "import json;print(json.loads(open('$O/cur_$i.json').read().strip().splitlines()[-1])['value'])") r4 $(python3 -c "import json;print(json.loads(open('$O/r4_$i.json').read().strip().splitlines()[-1])['value'])")
done
