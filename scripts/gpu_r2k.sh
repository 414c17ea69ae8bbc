set -o pipefail
mkdir -p gpurun_out/r2k
timeout -k 10 600 python -u -m pytest tests/ops/test_convbn_gpu.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2k/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r2k/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2k/amoeba.log 2>&1 || exit 1
tail -1 gpurun_out/r2k/amoeba.log | cut -c1-300
bash scripts/profile_bench.sh amoeba_r2k --model amoebanet --gpus 1 --steps 4 --warmup 2 || exit 1
head -40 gpurun_out/prof_amoeba_r2k/summary.md
