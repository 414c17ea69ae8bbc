# Final round-4 tree: whole GPU suite, then the default bench twice (U-Net headline with
# in-place transform refresh, AmoebaNet with captured cells, ResNet, re-tuned plans), and
# AmoebaNet n8m32 stages 5-6 with / without the recompute lane.
set -o pipefail
out=gpurun_out/r4aa
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "^E  \|Error" $out/gpu_tests.log | head -60; exit 1; }
for rep in 1 2; do
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_$rep.json 2> $out/bench_$rep.err || { tail -20 $out/bench_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$out/bench_$rep.json'));print('unet', d['value'], 'base', d['baseline']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'], d['resnet101'].get('baseline',{}).get('value'))"
done
timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6 --graph-cells --lanes on > $out/ab_s56_lanes.log 2>&1 || { tail -20 $out/ab_s56_lanes.log; exit 1; }
grep '"stage"' $out/ab_s56_lanes.log
timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6 --graph-cells > $out/ab_s56.log 2>&1 || { tail -20 $out/ab_s56.log; exit 1; }
grep '"stage"' $out/ab_s56.log
