# Round 3: shared duplicate pools + grouped ops + fused ResNet tests; AmoebaNet A/B of pool
# sharing; ResNet-101 pipeline-1 kernel tables (torch.profiler), fused and plain.
set -o pipefail
out=gpurun_out/r3z
mkdir -p $out
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/models/test_resnet_fused_gpu.py tests/ops/test_group_convbn_gpu.py tests/test_step_graph.py tests/models/test_amoebanet_streams.py tests/test_overlap_recompute.py > $out/tests.log 2>&1; rc=$?
tail -3 $out/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
run() {
  tag=$1; shift
  e=$1; shift; env $e timeout -k 10 300 python bench.py --model amoebanet --steps 5 --warmup 2 --sections none "$@" > $out/amoeba_$tag.json 2> $out/amoeba_$tag.err || { tail -20 $out/amoeba_$tag.err; return 1; }
  echo "$tag $(cut -c1-150 $out/amoeba_$tag.json)"
}
run share TGPIPE_SHARE_POOLS=1 || exit 1
run noshare TGPIPE_SHARE_POOLS=0 || exit 1
run share2 TGPIPE_SHARE_POOLS=1 || exit 1
PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py > $out/resnet_fused_table.txt 2> $out/resnet_fused_table.err; echo "fused rc=$?"; head -3 $out/resnet_fused_table.txt
PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py --plain > $out/resnet_plain_table.txt 2> $out/resnet_plain_table.err; echo "plain rc=$?"; head -3 $out/resnet_plain_table.txt
exit 0
