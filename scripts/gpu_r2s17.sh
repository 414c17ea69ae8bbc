# AmoebaNet stream configurations (after the single-split accumulate fix) and the weight-
# gradient stream parity test.
set -o pipefail
mkdir -p gpurun_out/s17
timeout -k 10 400 python -u -m pytest tests/test_overlap_recompute.py -q --timeout 300 --timeout-method thread > gpurun_out/s17/tests.log 2>&1
rc=$?; tail -2 gpurun_out/s17/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/s17/tests.log | head -20; }
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" > gpurun_out/s17/$tag.log 2>&1 || { tail -20 gpurun_out/s17/$tag.log; exit 1; }
  echo "$tag: $(tail -1 gpurun_out/s17/$tag.log | cut -c1-150)"
}
run amoeba_streams --model amoebanet --steps 10 --warmup 3
run amoeba_streams_wgrad --model amoebanet --steps 10 --warmup 3 --wgrad-stream on
run amoeba_plain --model amoebanet --steps 10 --warmup 3 --cell-streams off
run amoeba_wgrad --model amoebanet --steps 10 --warmup 3 --cell-streams off --wgrad-stream on
