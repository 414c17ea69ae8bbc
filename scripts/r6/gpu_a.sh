#!/bin/bash
# r6a: the changed GPU tests (pre-split .data updates, cache budgets), then bench N=1 with
# the new gpipe section.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6a
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/ops/test_convbn_gpu.py -k "presplit" tests/ops/test_winograd_gpu.py::test_cache_budget_sizing_modes \
    tests/test_overlap_recompute.py > $out/tests.log 2>&1 \
  && tail -2 $out/tests.log \
  && timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.log
rc=$?
tail -3 $out/tests.log
tail -1 $out/bench.json
exit $rc
