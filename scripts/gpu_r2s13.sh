# Two-stream AmoebaNet cells and overlapped recomputation: parity tests, then benches.
set -o pipefail
mkdir -p gpurun_out/s13
timeout -k 10 500 python -u -m pytest tests/test_step_graph.py tests/test_overlap_recompute.py -q --timeout 300 --timeout-method thread > gpurun_out/s13/tests.log 2>&1
rc=$?; tail -3 gpurun_out/s13/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/s13/tests.log | head -30; }
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" > gpurun_out/s13/$tag.log 2>&1 || { tail -20 gpurun_out/s13/$tag.log; exit 1; }
  echo "$tag: $(tail -1 gpurun_out/s13/$tag.log | cut -c1-190)"
}
run unet_overlap --steps 20 --warmup 5 --overlap-recompute
run unet --steps 20 --warmup 5
run amoeba_streams --model amoebanet --steps 10 --warmup 3 --cell-streams
run amoeba_streams_graph --model amoebanet --steps 10 --warmup 3 --cell-streams --graph
run amoeba_overlap_graph --model amoebanet --steps 10 --warmup 3 --overlap-recompute --graph
run amoeba_all --model amoebanet --steps 10 --warmup 3 --overlap-recompute --cell-streams --graph
