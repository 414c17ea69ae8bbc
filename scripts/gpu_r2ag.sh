set -o pipefail
mkdir -p gpurun_out/r2ag
timeout -k 10 600 python -u -m pytest tests/ops/test_winograd_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2ag/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r2ag/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/wino_variants.py --variants 6 14 --iters 30 --shape 40 64 64 192 --shape 40 128 64 192 --shape 40 128 128 96 --shape 40 256 128 96 --shape 40 256 256 48 --shape 40 512 256 48 --shape 40 1024 1024 12 > gpurun_out/r2ag/wino.log 2>&1 || { tail gpurun_out/r2ag/wino.log; exit 1; }
grep shape gpurun_out/r2ag/wino.log | cut -c1-250
timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2ag/unet.log 2>&1 || exit 1
tail -1 gpurun_out/r2ag/unet.log | cut -c1-200
