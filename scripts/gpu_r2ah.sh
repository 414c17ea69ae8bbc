set -o pipefail
mkdir -p gpurun_out/r2ah
timeout -k 10 600 python -u -m pytest tests/ops/test_winograd_gpu.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2ah/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r2ah/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/wino_variants.py --variants 6 --iters 30 --shape 40 64 64 192 --shape 40 128 64 192 --shape 40 128 128 96 --shape 40 256 256 48 > gpurun_out/r2ah/wino.log 2>&1 || { tail gpurun_out/r2ah/wino.log; exit 1; }
grep shape gpurun_out/r2ah/wino.log | cut -c1-120
timeout -k 10 300 python -u benchmarks/wgrad_variants.py --help > /dev/null 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2ah/unet.log 2>&1 || exit 1
tail -1 gpurun_out/r2ah/unet.log | cut -c1-200
bash scripts/profile_bench.sh unet_r2ah --gpus 1 --steps 4 --warmup 2 || exit 1
head -24 gpurun_out/prof_unet_r2ah/summary.md | tail -14
