# Weight-gradient stream on by default for one-GPU AmoebaNet: parity tests + default bench.
set -o pipefail
mkdir -p gpurun_out/s22
timeout -k 10 500 python -u -m pytest tests/test_overlap_recompute.py tests/test_step_graph.py -q --timeout 300 --timeout-method thread > gpurun_out/s22/tests.log 2>&1
rc=$?; tail -2 gpurun_out/s22/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/s22/tests.log | head -20; exit 1; }
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 > gpurun_out/s22/amoeba.log 2>&1 || { tail -20 gpurun_out/s22/amoeba.log; exit 1; }
echo "amoeba: $(tail -1 gpurun_out/s22/amoeba.log | cut -c1-200)"
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 --wgrad-stream off > gpurun_out/s22/amoeba_nowg.log 2>&1 || { tail -20 gpurun_out/s22/amoeba_nowg.log; exit 1; }
echo "amoeba_nowg: $(tail -1 gpurun_out/s22/amoeba_nowg.log | cut -c1-200)"
