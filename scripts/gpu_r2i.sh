set -o pipefail
mkdir -p gpurun_out/r2i
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/ops/test_winograd_gpu.py tests/ops/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2i/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r2i/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/kernel_bench.py --out gpurun_out/r2i/kernel_bench.json > gpurun_out/r2i/kb.log 2>&1 || { tail gpurun_out/r2i/kb.log; exit 1; }
grep dbn_bn gpurun_out/r2i/kb.log
