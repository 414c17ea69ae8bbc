set -o pipefail
mkdir -p gpurun_out/r2z
timeout -k 10 600 python -u -m pytest tests/ops/test_convbn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2z/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2z/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/convgemm_sweep.py --out gpurun_out/r2z/sweep.json > gpurun_out/r2z/sweep.log 2>&1 || { tail gpurun_out/r2z/sweep.log; exit 1; }
timeout -k 10 400 env TGPIPE_CG_DB=0 python -u benchmarks/convbn_bench.py --micro-batch 20 --out gpurun_out/r2z/convbn_bench_n20.json > gpurun_out/r2z/cb.log 2>&1 || { tail gpurun_out/r2z/cb.log; exit 1; }
tail -1 gpurun_out/r2z/cb.log
timeout -k 10 400 python -u benchmarks/tune_plans.py --out gpurun_out/r2z/conv_gemm_mi355x.txt > gpurun_out/r2z/tune.log 2>&1 || { tail gpurun_out/r2z/tune.log; exit 1; }
tail -1 gpurun_out/r2z/tune.log
timeout -k 10 300 env TGPIPE_CG_DB=gpurun_out/r2z/conv_gemm_mi355x.txt python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2z/amoeba.log 2>&1 || exit 1
tail -1 gpurun_out/r2z/amoeba.log | cut -c1-250
