# Whole-step hipGraph capture: GPU test, AmoebaNet bench eager and graphed (conflict-free
# K-major LDS image in the implicit-GEMM kernels).
set -o pipefail
mkdir -p gpurun_out/s9
timeout -k 10 300 python -u -m pytest tests/test_step_graph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s9/tests.log 2>&1
rc=$?; tail -3 gpurun_out/s9/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/s9/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 > gpurun_out/s9/amoeba.log 2>&1 || { tail -20 gpurun_out/s9/amoeba.log; exit 1; }
grep 'warmup step 1/' gpurun_out/s9/amoeba.log; tail -1 gpurun_out/s9/amoeba.log | cut -c1-250
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 --graph > gpurun_out/s9/amoeba_graph.log 2>&1 || { tail -20 gpurun_out/s9/amoeba_graph.log; exit 1; }
grep 'warmup step' gpurun_out/s9/amoeba_graph.log; tail -1 gpurun_out/s9/amoeba_graph.log | cut -c1-250
