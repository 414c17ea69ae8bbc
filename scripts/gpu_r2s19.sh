# Per-stream side streams for the AmoebaNet cells: parity tests, AmoebaNet streams with and
# without the recompute lane.
set -o pipefail
mkdir -p gpurun_out/s19
timeout -k 10 500 python -u -m pytest tests/test_overlap_recompute.py tests/test_step_graph.py -q --timeout 300 --timeout-method thread > gpurun_out/s19/tests.log 2>&1
rc=$?; tail -2 gpurun_out/s19/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/s19/tests.log | head -20; exit 1; }
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" > gpurun_out/s19/$tag.log 2>&1 || { tail -20 gpurun_out/s19/$tag.log; exit 1; }
  echo "$tag: $(tail -1 gpurun_out/s19/$tag.log | cut -c1-150)"
}
run amoeba_default --model amoebanet --steps 10 --warmup 3
run amoeba_overlap --model amoebanet --steps 10 --warmup 3 --overlap-recompute on
