# Round 2: fused AmoebaNet conv/BN kernels: numerics, then a short AmoebaNet bench.
set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 600 python -u -m pytest tests/ops/test_convbn_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2b/test_convbn.log 2>&1
rc=$?; tail -40 gpurun_out/r2b/test_convbn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 3 --warmup 2 > gpurun_out/r2b/amoeba.log 2>&1 || { tail -30 gpurun_out/r2b/amoeba.log; exit 1; }
tail -1 gpurun_out/r2b/amoeba.log | cut -c1-400
