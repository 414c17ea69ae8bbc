set -o pipefail
mkdir -p gpurun_out/r2l
timeout -k 10 600 python -u -m pytest tests/ops/test_convbn_gpu.py tests/test_gpu_pipeline.py tests/test_deferred_batch_norm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2l/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r2l/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u benchmarks/tune_plans.py --out gpurun_out/r2l/conv_gemm_mi355x.txt > gpurun_out/r2l/tune.log 2>&1 || { tail gpurun_out/r2l/tune.log; exit 1; }
cat gpurun_out/r2l/tune.log
timeout -k 10 300 env TGPIPE_CG_DB=gpurun_out/r2l/conv_gemm_mi355x.txt python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2l/amoeba.log 2>&1 || exit 1
grep "warmup step 1/" gpurun_out/r2l/amoeba.log; tail -1 gpurun_out/r2l/amoeba.log | cut -c1-300
