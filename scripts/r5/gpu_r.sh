#!/bin/bash
# Round 5: fitted split-K models for the F(4x4) kernels -- numerics, sweep, bench N=1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5r
timeout -k 10 300 python -u -m pytest tests/ops/test_winograd_gpu.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r5r/wino_tests.log 2>&1 \
  && timeout -k 10 420 python -u benchmarks/split_sweep.py --out gpurun_out/r5r/split_sweep.json \
    > gpurun_out/r5r/split_sweep.log 2>&1 \
  && timeout -k 10 600 python -u bench.py > gpurun_out/r5r/bench.json 2> gpurun_out/r5r/bench.log
rc=$?
tail -2 gpurun_out/r5r/wino_tests.log
cat gpurun_out/r5r/bench.json
exit $rc
