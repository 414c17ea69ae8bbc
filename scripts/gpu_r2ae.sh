set -o pipefail
mkdir -p gpurun_out/r2ae
timeout -k 10 600 python -u -m pytest tests/ops/test_unet_ops_gpu.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2ae/tests.log 2>&1
rc=$?; tail -15 gpurun_out/r2ae/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2ae/unet.log 2>&1 || exit 1
tail -1 gpurun_out/r2ae/unet.log | cut -c1-200
