# Round 3: grouped ReLU-Conv-BN (normal cells' node-0 triplets as one GEMM): tests, then
# AmoebaNet n1m32 A/B (grouped / ungrouped / grouped), separate processes.
set -o pipefail
out=gpurun_out/r3w
mkdir -p $out
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/ops/test_group_convbn_gpu.py tests/models/test_resnet_fused_gpu.py tests/ops/test_deferred_wgrad_gpu.py tests/test_step_graph.py > $out/tests.log 2>&1; rc=$?
tail -3 $out/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
run() {
  tag=$1; shift
  e=$1; shift; env $e timeout -k 10 300 python bench.py --model amoebanet --steps 5 --warmup 2 --sections none "$@" > $out/amoeba_$tag.json 2> $out/amoeba_$tag.err || { tail -20 $out/amoeba_$tag.err; return 1; }
  echo "$tag $(cut -c1-150 $out/amoeba_$tag.json)"
}
run group TGPIPE_GROUP_CONVBN=1 || exit 1
run nogroup TGPIPE_GROUP_CONVBN=0 || exit 1
run group2 TGPIPE_GROUP_CONVBN=1 || exit 1
run eager_group TGPIPE_GROUP_CONVBN=1 --graph off || exit 1
