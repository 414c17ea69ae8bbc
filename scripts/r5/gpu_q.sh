#!/bin/bash
# Round 5: full GPU test suite (striped rehearsal, graph-cell accumulation tests), smoke,
# then the F(4x4) split-K sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5q
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r5q/gpu_tests.log 2>&1 \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5q/smoke.log 2>&1 \
  && timeout -k 10 400 python -u benchmarks/split_sweep.py --out gpurun_out/r5q/split_sweep.json \
    > gpurun_out/r5q/split_sweep.log 2>&1
rc=$?
tail -3 gpurun_out/r5q/gpu_tests.log
exit $rc
