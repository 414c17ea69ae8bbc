set -o pipefail
mkdir -p gpurun_out/r2ac
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q -k "exits_cleanly" --timeout 200 --timeout-method thread > gpurun_out/r2ac/test.log 2>&1
rc=$?; tail -15 gpurun_out/r2ac/test.log
timeout -k 10 300 python -u benchmarks/amoeba_op_profile.py --chunks 4 --batch 80 --rows 5 > gpurun_out/r2ac/ops.log 2>&1
echo "profile rc=$?"
grep -A7 "^aten::" gpurun_out/r2ac/ops.log | head -120
