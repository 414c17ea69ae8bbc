# Stream-concurrency defaults: bench defaults (U-Net, AmoebaNet) and AmoebaNet ablations.
set -o pipefail
mkdir -p gpurun_out/s14
timeout -k 10 500 python -u -m pytest tests/test_step_graph.py tests/test_overlap_recompute.py -q --timeout 300 --timeout-method thread > gpurun_out/s14/tests.log 2>&1
rc=$?; tail -2 gpurun_out/s14/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/s14/tests.log | head -30; exit 1; }
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" > gpurun_out/s14/$tag.log 2>&1 || { tail -20 gpurun_out/s14/$tag.log; exit 1; }
  echo "$tag: $(tail -1 gpurun_out/s14/$tag.log | cut -c1-190)"
}
run unet_default --steps 20 --warmup 5
run amoeba_default --model amoebanet --steps 10 --warmup 3
run amoeba_streams_only --model amoebanet --steps 10 --warmup 3 --overlap-recompute off
run amoeba_graph --model amoebanet --steps 10 --warmup 3 --graph
