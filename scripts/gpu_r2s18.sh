# Forward lanes (stateless one-rank partitions) on top of the recompute lane: parity tests,
# U-Net p1 bench, AmoebaNet default bench (stateful: unchanged path).
set -o pipefail
mkdir -p gpurun_out/s18
timeout -k 10 500 python -u -m pytest tests/test_overlap_recompute.py tests/test_step_graph.py tests/test_gpu_pipeline.py -q --timeout 300 --timeout-method thread > gpurun_out/s18/tests.log 2>&1
rc=$?; tail -2 gpurun_out/s18/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/s18/tests.log | head -20; exit 1; }
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" > gpurun_out/s18/$tag.log 2>&1 || { tail -20 gpurun_out/s18/$tag.log; exit 1; }
  echo "$tag: $(tail -1 gpurun_out/s18/$tag.log | cut -c1-150)"
}
run unet_default --steps 20 --warmup 5
run unet_fwd_lanes --steps 20 --warmup 5 --overlap-forward on
run unet_one_stream --steps 20 --warmup 5 --overlap-recompute off
run amoeba_default --model amoebanet --steps 10 --warmup 3
