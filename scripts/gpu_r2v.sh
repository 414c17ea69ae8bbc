set -o pipefail
mkdir -p gpurun_out/r2v
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2v/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2v/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2v/unet.log 2>&1 || exit 1
grep 'warmup step 1/' gpurun_out/r2v/unet.log; tail -1 gpurun_out/r2v/unet.log | cut -c1-200
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2v/amoeba.log 2>&1 || exit 1
grep 'warmup step 1/' gpurun_out/r2v/amoeba.log; tail -1 gpurun_out/r2v/amoeba.log | cut -c1-200
bash scripts/profile_bench.sh amoeba_r2v --model amoebanet --gpus 1 --steps 4 --warmup 2 || exit 1
bash scripts/profile_bench.sh unet_r2v --gpus 1 --steps 4 --warmup 2 || exit 1
head -8 gpurun_out/prof_amoeba_r2v/summary.md; head -8 gpurun_out/prof_unet_r2v/summary.md
