# Small-plane memory-bound kernels (multi-plane pools and split reduction, unrolled 7^2
# BatchNorm passes) and the 64x64 two-sub-stage GEMM tile: numerics, sweep, stage 6, bench.
set -o pipefail
out=gpurun_out/r4q
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/ops/test_convbn_gpu.py tests/ops/test_group_convbn_gpu.py tests/ops/test_deferred_wgrad_gpu.py tests/ops/test_lib_dgrad_gpu.py tests/models/test_resnet_fused_gpu.py -q -x --timeout 120 --timeout-method thread > $out/conv_tests.log 2>&1 || { tail -30 $out/conv_tests.log; exit 1; }
tail -2 $out/conv_tests.log
timeout -k 10 300 python -u benchmarks/convgemm_sweep.py --micro-batch 40 --out $out/convgemm_sweep_n40.json > $out/sweep.log 2>&1 || { tail -20 $out/sweep.log; exit 1; }
timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 6 --graph-cells > $out/harness_s6.log 2>&1 || { tail -20 $out/harness_s6.log; exit 1; }
grep '"stage"' $out/harness_s6.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_amoeba_s6 -o run -- python3 benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 6 --graph-cells --steps 2 > $out/prof_amoeba_s6.log 2>&1 || { tail -20 $out/prof_amoeba_s6.log; exit 1; }
timeout -k 10 600 python -u bench.py --gpus 1 --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('unet', d['value'], 'base', d['baseline']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'], d['resnet101'].get('baseline',{}).get('value'))"
