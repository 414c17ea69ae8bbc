set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/bench_p1_f4.log 2>&1 || exit 1
tail -1 gpurun_out/bench_p1_f4.log
timeout -k 10 400 python benchmarks/layer_profile.py --model unet --micro-batch 16 --out gpurun_out/unet_layer_profile_f4.json > gpurun_out/layer_prof_f4.log 2>&1 || exit 1
bash scripts/profile_bench.sh unet_p1_f4 --gpus 1 --steps 4 --warmup 2 || exit 1
echo DONE
