set -o pipefail
mkdir -p gpurun_out/r2u
timeout -k 10 600 python -u -m pytest tests/ops/test_convbn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2u/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r2u/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/convgemm_sweep.py --out gpurun_out/r2u/sweep.json > gpurun_out/r2u/sweep.log 2>&1 || { tail gpurun_out/r2u/sweep.log; exit 1; }
