set -o pipefail
mkdir -p gpurun_out/r2an
timeout -k 10 900 python -u -m pytest tests/ops/test_convbn_gpu.py tests/ops/test_unet_ops_gpu.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2an/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2an/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r2an/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2an/amoeba.log 2>&1 || { tail -20 gpurun_out/r2an/amoeba.log; exit 1; }
grep 'warmup step' gpurun_out/r2an/amoeba.log; tail -1 gpurun_out/r2an/amoeba.log | cut -c1-200
