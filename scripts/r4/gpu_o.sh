# Interleaved implicit-GEMM loads spread over the first half of each sub-stage: numerics,
# mb-40 sweep / per-shape table, AmoebaNet n8m32 stage 6 and the bench.
set -o pipefail
out=gpurun_out/r4o
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/ops/test_convbn_gpu.py tests/ops/test_group_convbn_gpu.py -q -x --timeout 120 --timeout-method thread > $out/conv_tests.log 2>&1 || { tail -30 $out/conv_tests.log; exit 1; }
tail -2 $out/conv_tests.log
timeout -k 10 300 python -u benchmarks/convgemm_sweep.py --micro-batch 40 --out $out/convgemm_sweep_n40.json > $out/sweep.log 2>&1 || { tail -20 $out/sweep.log; exit 1; }
timeout -k 10 300 python -u benchmarks/convbn_bench.py --micro-batch 40 --out $out/convbn_bench_n40.json > $out/convbn_bench.log 2>&1 || { tail -20 $out/convbn_bench.log; exit 1; }
tail -1 $out/convbn_bench.log
timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 6 --graph-cells > $out/harness_s6.log 2>&1 || { tail -20 $out/harness_s6.log; exit 1; }
grep '"stage"' $out/harness_s6.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('unet', d['value'], 'base', d['baseline']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'], d['resnet101'].get('baseline',{}).get('value'))"
