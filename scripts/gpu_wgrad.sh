set -o pipefail
timeout -k 10 300 python -u -m pytest tests/ops/test_winograd_gpu.py -x -q --timeout 120 --timeout-method thread -k "f4" > gpurun_out/f4_wgrad_tests.log 2>&1 || { tail -30 gpurun_out/f4_wgrad_tests.log; exit 1; }
tail -2 gpurun_out/f4_wgrad_tests.log
timeout -k 10 300 python benchmarks/wgrad_variants.py --out gpurun_out/wgrad_f4.json > gpurun_out/wgrad_f4.log 2>&1 || { tail -20 gpurun_out/wgrad_f4.log; exit 1; }
cat gpurun_out/wgrad_f4.log
timeout -k 10 300 python benchmarks/wino_variants.py --out gpurun_out/wino_f4_vec.json > gpurun_out/wino_f4_vec.log 2>&1 || { tail -20 gpurun_out/wino_f4_vec.log; exit 1; }
cat gpurun_out/wino_f4_vec.log
