# Captured cells (graph_cells): targeted tests first, then the whole GPU suite.
set -o pipefail
out=gpurun_out/r4b
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_segments.py tests/test_overlap_recompute.py tests/distributed/test_shared_gpu_rehearsal.py \
  tests/ops/test_winograd_gpu.py -k "segments or graph or overlap or rehearsal or retain or Overlapped or overlapped" \
  > $out/seg_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $out/seg_tests.log | tail -40
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -5 $out/gpu_tests.log
exit $rc
