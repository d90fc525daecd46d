# PMC traffic refresh after the XCD-grouped attention: C2-bf16, C5, C5 mixed
set -euo pipefail
OUT=gpurun_out/pmcy; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/pmc_bench.sh $OUT/pmc_c2bf16 --precision bf16 > $OUT/pmc_c2bf16.log 2>&1
bash tools/pmc_bench.sh $OUT/pmc_c5 --size 1280 --batch 8 > $OUT/pmc_c5.log 2>&1
bash tools/pmc_bench.sh $OUT/pmc_c5mixed --size 1280 --batch 8 --stream mixed > $OUT/pmc_c5mixed.log 2>&1
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
echo done
