# Round 3: deferred split weight gradients (slabs) + fused split-reduce/BN-stats forward +
# fused ResNet Conv-BN-ReLU runs: numerics tests, AmoebaNet n1m32 A/B (deferral on / off /
# on, separate processes), ResNet-101 pipeline-1 fused vs plain.
set -o pipefail
out=gpurun_out/r3s
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ops/test_deferred_wgrad_gpu.py tests/models/test_resnet_fused_gpu.py tests/ops/test_convbn_gpu.py tests/test_step_graph.py tests/test_overlap_recompute.py > $out/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for tag in on off on2; do
  v=1; [ $tag = off ] && v=0
  TGPIPE_DEFERRED_WGRAD=$v timeout -k 10 300 python bench.py --model amoebanet --steps 5 --warmup 2 --sections none > $out/amoeba_$tag.json 2> $out/amoeba_$tag.err || { tail -20 $out/amoeba_$tag.err; exit 1; }
  echo "$tag $(cut -c1-200 $out/amoeba_$tag.json)"
done
cd benchmarks
for v in fused plain; do
  f=""; [ $v = plain ] && f=--plain
  timeout -k 10 300 python resnet101_speed.py pipeline-1 $f --epochs 3 --skip-epochs 1 --dataset-size 2200 --json > ../$out/resnet_p1_$v.json 2> ../$out/resnet_p1_$v.err || { tail -20 ../$out/resnet_p1_$v.err; exit 1; }
  echo "$v $(cat ../$out/resnet_p1_$v.json)"
done
