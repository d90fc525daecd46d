# kernel durations of the bs1 forward with the in-launch split-K combine vs the separate reduce launch
set -o pipefail
O=gpurun_out/r5k; mkdir -p $O && export TMPDIR=/tmp
for v in plain sep; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o bs1 -- python3 tools/bs1_ab.py --reps 20 --rounds 1 --variants $v:-1:16:8 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  grep variant $O/$v.log | cut -c1-200
done
