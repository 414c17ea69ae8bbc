set -o pipefail
mkdir -p gpurun_out/r2ad
timeout -k 10 600 python -u -m pytest tests/ops/test_convbn_gpu.py tests/test_gpu_pipeline.py tests/test_deferred_batch_norm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2ad/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2ad/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2ad/amoeba.log 2>&1 || exit 1
tail -1 gpurun_out/r2ad/amoeba.log | cut -c1-200
