# Winograd F(4x4) transform rates on the C2 shapes against a same-bytes copy
set -o pipefail
O=gpurun_out/r5i; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/microbench/wino_tf.py --reps 20 --out $O/wino_tf.json > $O/wino_tf.log 2>&1 || { tail -20 $O/wino_tf.log; exit 1; }
cat $O/wino_tf.log
