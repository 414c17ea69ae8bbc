#!/bin/bash
# r5au: full GPU suite on the final tree (re-timed plan tables), smoke, bench N=1 on the current tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5au
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > $out/gpu_tests.log 2>&1 \
  && tail -1 $out/gpu_tests.log \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 \
  && timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.log
rc=$?
tail -3 $out/gpu_tests.log
cat $out/bench.json
exit $rc
