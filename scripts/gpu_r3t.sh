# Round 3: deferred weight-gradient slabs, fused split statistics, one-pass BatchNorm
# backward, fused ResNet Conv-BN-ReLU runs: tests; AmoebaNet n1m32 A/B (separate processes);
# ResNet-101 pipeline-1 fused vs plain; rocprofv3 kernel trace of AmoebaNet (eager).
set -o pipefail
out=gpurun_out/r3t
mkdir -p $out
PYTHONPATH=. timeout -k 10 200 python benchmarks/diag/resnet_fused_diag.py 2>&1 | grep composite
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/ops/test_deferred_wgrad_gpu.py tests/models/test_resnet_fused_gpu.py tests/ops/test_convbn_gpu.py tests/test_step_graph.py tests/test_overlap_recompute.py > $out/tests.log 2>&1; rc=$?
tail -3 $out/tests.log
# (a failing numerics test does not stop the measurements; a fault or hang does)
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
run() {  # tag, env..., then bench args
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --model amoebanet --steps 5 --warmup 2 --sections none > $out/amoeba_$tag.json 2> $out/amoeba_$tag.err || { tail -20 $out/amoeba_$tag.err; return 1; }
  echo "$tag $(cut -c1-150 $out/amoeba_$tag.json)"
}
run all TGPIPE_DEFERRED_WGRAD=1 || exit 1
run noslab TGPIPE_DEFERRED_WGRAD=0 || exit 1
run twopass TGPIPE_BN_BWD_ONEPASS=0 || exit 1
run all2 TGPIPE_DEFERRED_WGRAD=1 || exit 1
cd benchmarks
for v in fused plain; do
  f=""; [ $v = plain ] && f=--plain
  timeout -k 10 300 python resnet101_speed.py pipeline-1 $f --epochs 3 --skip-epochs 1 --dataset-size 2200 --json > ../$out/resnet_p1_$v.json 2> ../$out/resnet_p1_$v.err || { tail -20 ../$out/resnet_p1_$v.err; exit 1; }
  echo "$v $(cat ../$out/resnet_p1_$v.json)"
done
cd ..
bash scripts/profile_bench.sh amoeba_r3t --model amoebanet --graph off --steps 3 --warmup 2 --sections none || exit 1
head -30 gpurun_out/prof_amoeba_r3t/summary.md
