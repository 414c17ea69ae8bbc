# Final tree: full GPU test suite, smoke, default U-Net p1 bench.
set -o pipefail
mkdir -p gpurun_out/final2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final2/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/final2/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/final2/gpu_tests.log | head -20; exit 1; }
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/final2/smoke.log 2>&1 || { tail -20 gpurun_out/final2/smoke.log; exit 1; }
tail -1 gpurun_out/final2/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final2/unet.log 2>&1 || { tail -20 gpurun_out/final2/unet.log; exit 1; }
echo "unet: $(tail -1 gpurun_out/final2/unet.log | cut -c1-200)"
