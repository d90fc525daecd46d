# PMC traffic refresh after the XCD-grouped attention (C2 and C3), then the C2 line that reads it
set -euo pipefail
OUT=gpurun_out/pmcx; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/pmc_bench.sh $OUT/pmc_c2 > $OUT/pmc_c2.log 2>&1
bash tools/pmc_bench.sh $OUT/pmc_c3 --preset r18vd --precision bf16 --batch 256 > $OUT/pmc_c3.log 2>&1
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
timeout -k 10 600 python3 -u bench.py > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | cut -c1-200
