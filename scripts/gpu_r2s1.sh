# Session re-entry check: full GPU test suite, smoke, U-Net p1 and AmoebaNet n1m32 benches.
set -o pipefail
mkdir -p gpurun_out/s1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s1/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s1/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/s1/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/s1/smoke.log 2>&1 || { tail -20 gpurun_out/s1/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s1/unet.log 2>&1 || { tail -20 gpurun_out/s1/unet.log; exit 1; }
tail -1 gpurun_out/s1/unet.log | cut -c1-250
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 > gpurun_out/s1/amoeba.log 2>&1 || { tail -20 gpurun_out/s1/amoeba.log; exit 1; }
grep 'warmup step' gpurun_out/s1/amoeba.log; tail -1 gpurun_out/s1/amoeba.log | cut -c1-250
