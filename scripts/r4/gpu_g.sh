# Whole GPU suite, the offline plan tuner (new tables), default bench, AmoebaNet harness
# with three-stream captured cells.
set -o pipefail
out=gpurun_out/r4g
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -4 $out/gpu_tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "^E  \|Error" $out/gpu_tests.log | head -60; exit 1; }
timeout -k 10 900 python -u benchmarks/tune_plans.py --out $out/conv_gemm_mi355x.txt --lib-out $out/lib_dgrad_mi355x.txt > $out/tune.log 2>&1; echo "tune rc=$?"; tail -12 $out/tune.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6 --graph-cells > $out/harness_amoeba_gc3.log 2>&1 || { tail -20 $out/harness_amoeba_gc3.log; exit 1; }
grep stage $out/harness_amoeba_gc3.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 10 --warmup 4 --graph-cells on --sections none > $out/bench_unet_gc.json 2> $out/bench_unet_gc.err || { tail -20 $out/bench_unet_gc.err; exit 1; }
cat $out/bench_unet_gc.json
