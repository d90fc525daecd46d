# whole-request /detect path: repeated image (exact glyph-mask repeats) and jittered boxes (class memo only)
set -o pipefail
O=gpurun_out/r5n; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_jpeg.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python3 -u tools/detect_path.py --iters 100 > $O/detect_path.json 2> $O/dp.err || { tail -5 $O/dp.err; exit 1; }
cut -c180-600 $O/detect_path.json
timeout -k 10 300 python3 -u tools/detect_path.py --iters 100 --jitter > $O/detect_path_jitter.json 2> $O/dpj.err || { tail -5 $O/dpj.err; exit 1; }
cut -c180-600 $O/detect_path_jitter.json
