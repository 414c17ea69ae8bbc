set -o pipefail
mkdir -p gpurun_out/r2g
for k in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2g/unet_run$k.log 2>&1 || exit 1
  grep 'warmup step 1' gpurun_out/r2g/unet_run$k.log; tail -1 gpurun_out/r2g/unet_run$k.log | cut -c1-200
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2g/gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r2g/gpu_tests.log; exit $rc
