set -o pipefail
mkdir -p gpurun_out/r2w
timeout -k 10 600 python -u -m pytest tests/ops/test_convbn_gpu.py -x -q -k "avgpool or fused" --timeout 120 --timeout-method thread > gpurun_out/r2w/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r2w/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2w/amoeba.log 2>&1 || exit 1
tail -1 gpurun_out/r2w/amoeba.log | cut -c1-200
bash scripts/profile_bench.sh amoeba_r2w --model amoebanet --gpus 1 --steps 4 --warmup 2 || exit 1
grep -E "avgpool|add<float>" gpurun_out/prof_amoeba_r2w/summary.md | cut -c1-150
