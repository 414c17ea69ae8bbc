# Round 3 re-entry check on the current tree: GPU tests, default bench (U-Net p1 headline +
# no-GPipe baseline + AmoebaNet n1m32 sections).
set -o pipefail
out=gpurun_out/r3q
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 5 --warmup 2 > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
