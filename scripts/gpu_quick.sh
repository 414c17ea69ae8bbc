# GPU tests + 1-GPU bench + rocprof summary (tag in $1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/bench_p1.log 2>&1 || { tail -20 gpurun_out/bench_p1.log; exit 1; }
tail -1 gpurun_out/bench_p1.log | cut -c1-300
bash scripts/profile_bench.sh ${1:-unet_p1} --gpus 1 --steps 4 --warmup 2 || exit 1
head -30 gpurun_out/prof_${1:-unet_p1}/summary.md
