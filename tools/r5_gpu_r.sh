# C2 with two micro-batch streams (16 + 16 images, interleaved block by block) against one stream, alternating
set -o pipefail
O=gpurun_out/r5r; mkdir -p $O && export TMPDIR=/tmp
B="python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --latency-iters 0 --no-events"
for i in 1 2; do
  for v in "one:" "two:--microbatches 2" "two_s2:--microbatches 2 --stagger 2" "two_s4:--microbatches 2 --stagger 4"; do
    name=${v%%:*}; args=${v#*:}
    timeout -k 10 300 $B $args > $O/${name}_$i.json 2> $O/${name}_$i.err || { tail -5 $O/${name}_$i.err; exit 1; }
    echo $name $i $(python3 -c "import json;print(json.loads(open('$O/${name}_$i.json').read().strip().splitlines()[-1])['value'])")
  done
done
