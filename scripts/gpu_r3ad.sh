# Round 3: element-gathered GEMM columns spread over the lanes (coalesced 7x7 / tap
# gathers): every tile config vs fp64, then AmoebaNet n1m32 A/B and per-shape timings.
set -o pipefail
out=gpurun_out/r3ad
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ops/test_convbn_gpu.py tests/ops/test_group_convbn_gpu.py tests/models/test_resnet_fused_gpu.py > $out/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
run() {
  tag=$1; shift
  e=$1; shift; env $e timeout -k 10 300 python bench.py --model amoebanet --steps 5 --warmup 2 --sections none "$@" > $out/amoeba_$tag.json 2> $out/amoeba_$tag.err || { tail -20 $out/amoeba_$tag.err; return 1; }
  echo "$tag $(cut -c1-150 $out/amoeba_$tag.json)"
}
run spread TGPIPE_CG_SPREAD=1 || exit 1
run quads TGPIPE_CG_SPREAD=0 || exit 1
run spread2 TGPIPE_CG_SPREAD=1 || exit 1
TGPIPE_CG_SPREAD=1 timeout -k 10 400 python benchmarks/convbn_bench.py --micro-batch 20 --out $out/convbn_spread.json > $out/convbn_spread.log 2>&1 || { tail -5 $out/convbn_spread.log; exit 1; }
TGPIPE_CG_SPREAD=0 timeout -k 10 400 python benchmarks/convbn_bench.py --micro-batch 20 --out $out/convbn_quads.json > $out/convbn_quads.log 2>&1 || { tail -5 $out/convbn_quads.log; exit 1; }
tail -3 $out/convbn_spread.log $out/convbn_quads.log
# three-stream capture with the side streams created before the capture
TGPIPE_CAPTURE_CELL_STREAMS=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_step_graph.py > $out/capture3_tests.log 2>&1; rc=$?
echo "capture3 tests rc=$rc"; tail -2 $out/capture3_tests.log
if [ $rc -eq 0 ]; then
  run cap3 "TGPIPE_CAPTURE_CELL_STREAMS=3" || exit 1
fi
