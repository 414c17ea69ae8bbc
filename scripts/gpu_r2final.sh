# End-of-session check on the committed tree: full GPU test suite, smoke, default benches
# (U-Net p1 = the driver's BENCH config; AmoebaNet n1m32), kernel traces of both.
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/final/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/final/gpu_tests.log | head -20; exit 1; }
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/unet.log 2>&1 || { tail -20 gpurun_out/final/unet.log; exit 1; }
echo "unet: $(tail -1 gpurun_out/final/unet.log | cut -c1-200)"
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 > gpurun_out/final/amoeba.log 2>&1 || { tail -20 gpurun_out/final/amoeba.log; exit 1; }
echo "amoeba: $(tail -1 gpurun_out/final/amoeba.log | cut -c1-200)"
bash scripts/profile_bench.sh unet_final --gpus 1 --steps 4 --warmup 2 || exit 1
bash scripts/profile_bench.sh amoeba_final --model amoebanet --gpus 1 --steps 3 --warmup 2 || exit 1
head -3 gpurun_out/prof_unet_final/summary.md | tail -1; head -3 gpurun_out/prof_amoeba_final/summary.md | tail -1
