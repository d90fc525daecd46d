#!/bin/bash
# Same-box A/B of this tree against the round-start tree built under _abtree/ (git archive <commit> | tar -x -C
# _abtree; python -m spotter_amd.build_ext there): C2 / C3 / C2-bf16 bench lines alternating, events off.
# .gpurunignore drops ./_abtree by default: narrow it to ./_abtree/spotter_amd/_build for the run.
set -euo pipefail
OUT=${1:-gpurun_out/abtree}; mkdir -p $OUT
B="python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --latency-iters 0 --no-events"
for r in 1 2; do
  for T in head base; do
    D=.; X=--no-input-supply  # (the round-start bench has no input-supply leg and no flag for it)
    [ $T = base ] && D=_abtree && X=
    for cfg in "c2:" "c3:--preset r18vd --precision bf16 --batch 256 --steps 10 --warmup 3" "c2bf16:--precision bf16"; do
      name=${cfg%%:*}; args=${cfg#*:}
      (cd $D && timeout -k 10 300 $B $X $args) > $OUT/${name}_${T}_$r.log 2>&1
      echo "$name $T $r $(grep -o '"value": [0-9.]*' $OUT/${name}_${T}_$r.log | head -1)"
    done
  done
done
