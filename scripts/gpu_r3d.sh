# Round 3 call d: batched-GEMM Winograd numerics + microbenchmark.
set -o pipefail
out=gpurun_out/r3d
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/ops/test_winograd_gpu.py -m gpu -x -q -k "batched" --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $out/tests.log | head -30; exit 1; }
timeout -k 10 300 python -u benchmarks/bg_bench.py --out $out/bg_bench.json > $out/bg_bench.log 2>&1 || { tail -20 $out/bg_bench.log; exit 1; }
cat $out/bg_bench.log | cut -c1-250
