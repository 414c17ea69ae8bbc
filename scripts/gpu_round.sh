# Full GPU check: tests, 1-GPU bench, kernel variant tables, rocprof summary of the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/bench_p1.log 2>&1 || { tail -20 gpurun_out/bench_p1.log; exit 1; }
tail -1 gpurun_out/bench_p1.log | cut -c1-300
timeout -k 10 300 python benchmarks/wino_variants.py --variants 2 4 5 --out gpurun_out/wino_f4_variants.json > gpurun_out/wino_f4_variants.log 2>&1 || exit 1
bash scripts/profile_bench.sh unet_p1 --gpus 1 --steps 4 --warmup 2 || exit 1
head -16 gpurun_out/prof_unet_p1/summary.md
timeout -k 10 400 python benchmarks/layer_profile.py --model unet --micro-batch 16 --out gpurun_out/unet_layer_profile_f4w.json > gpurun_out/layer_prof_f4w.log 2>&1 || exit 1
