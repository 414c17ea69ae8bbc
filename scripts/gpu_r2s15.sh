# Fast division in the implicit-GEMM gathers + stream concurrency (two-stream cells, recompute
# lanes, weight-gradient stream): parity tests, then benches.
set -o pipefail
mkdir -p gpurun_out/s15
timeout -k 10 600 python -u -m pytest tests/ops/test_convbn_gpu.py tests/test_step_graph.py tests/test_overlap_recompute.py -q --timeout 300 --timeout-method thread > gpurun_out/s15/tests.log 2>&1
rc=$?; tail -2 gpurun_out/s15/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/s15/tests.log | head -30; exit 1; }
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --gpus 1 "$@" > gpurun_out/s15/$tag.log 2>&1 || { tail -20 gpurun_out/s15/$tag.log; exit 1; }
  echo "$tag: $(tail -1 gpurun_out/s15/$tag.log | cut -c1-190)"
}
run amoeba_default --model amoebanet --steps 10 --warmup 3
run amoeba_no_wgrad_stream --model amoebanet --steps 10 --warmup 3 --wgrad-stream off
run unet_default --steps 20 --warmup 5
run unet_no_wgrad_stream --steps 20 --warmup 5 --wgrad-stream off
run amoeba_graph --model amoebanet --steps 10 --warmup 3 --graph
