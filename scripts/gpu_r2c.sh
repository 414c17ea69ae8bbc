# conv GEMM v2: numerics, per-shape timing, AmoebaNet bench
set -o pipefail
mkdir -p gpurun_out/r2c
timeout -k 10 600 python -u -m pytest tests/ops/test_convbn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2c/test_convbn.log 2>&1
rc=$?; tail -15 gpurun_out/r2c/test_convbn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/convbn_bench.py --micro-batch 20 --out gpurun_out/r2c/convbn_bench.json > gpurun_out/r2c/convbn_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r2c/convbn_bench.log
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 3 --warmup 2 > gpurun_out/r2c/amoeba.log 2>&1 || { tail -30 gpurun_out/r2c/amoeba.log; exit 1; }
tail -1 gpurun_out/r2c/amoeba.log | cut -c1-300
