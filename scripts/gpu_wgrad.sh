set -o pipefail
timeout -k 10 300 python -u -m pytest tests/ops/test_winograd_gpu.py -x -q --timeout 120 --timeout-method thread -k "f4_wgrad" > gpurun_out/f4_wgrad_tests.log 2>&1 || { tail -30 gpurun_out/f4_wgrad_tests.log; exit 1; }
tail -1 gpurun_out/f4_wgrad_tests.log
timeout -k 10 300 python benchmarks/wgrad_variants.py --out gpurun_out/wgrad_f4nf.json > gpurun_out/wgrad_f4nf.log 2>&1 || { tail -20 gpurun_out/wgrad_f4nf.log; exit 1; }
echo DONE
