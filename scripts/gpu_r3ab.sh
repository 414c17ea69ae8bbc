# Round 3: AmoebaNet cells on three streams (the two 1x7-7x1 chains after the grouped op
# side by side): parity tests, then n1m32 A/B 3 / 2 / 3 streams (graphed), 3 eager.
set -o pipefail
out=gpurun_out/r3ab
mkdir -p $out
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_step_graph.py tests/ops/test_group_convbn_gpu.py tests/ops/test_deferred_wgrad_gpu.py tests/test_overlap_recompute.py tests/models/test_amoebanet_streams.py > $out/tests.log 2>&1; rc=$?
tail -3 $out/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
run() {
  tag=$1; shift
  e=$1; shift; env $e timeout -k 10 300 python bench.py --model amoebanet --steps 5 --warmup 2 --sections none "$@" > $out/amoeba_$tag.json 2> $out/amoeba_$tag.err || { tail -20 $out/amoeba_$tag.err; return 1; }
  echo "$tag $(cut -c1-150 $out/amoeba_$tag.json)"
}
run g2 TGPIPE_CELL_STREAMS=2 || exit 1
run e3 TGPIPE_CELL_STREAMS=3 --graph off || exit 1
run e2 TGPIPE_CELL_STREAMS=2 --graph off || exit 1
run e3b TGPIPE_CELL_STREAMS=3 --graph off || exit 1
run g2b TGPIPE_CELL_STREAMS=2 || exit 1
