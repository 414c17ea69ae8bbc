set -o pipefail
out=gpurun_out/r4d
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_segments.py tests/distributed/test_shared_gpu_rehearsal.py tests/ops/test_lib_dgrad_gpu.py \
  > $out/seg_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $out/seg_tests.log | tail -30
[ $rc -eq 0 ] || { grep -B2 -A25 "^E   \|Error" $out/seg_tests.log | head -80; exit 1; }
timeout -k 10 300 python -u benchmarks/bg_bench.py --shapes "32,128,128,96;16,128,128,96;40,128,128,96;32,64,64,192;32,128,64,96;32,64,128,96" --out $out/bg_bench_128.json > $out/bg_bench.log 2>&1; echo "bg rc=$?"; tail -8 $out/bg_bench.log
for gc in "" "--graph-cells"; do
  timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 0 5 6 7 $gc > $out/harness_amoeba$gc.log 2>&1 || { echo "harness amoeba $gc failed"; tail -20 $out/harness_amoeba$gc.log; exit 1; }
  cat $out/harness_amoeba$gc.log
done
for gc in "" "--graph-cells"; do
  timeout -k 10 300 python -u benchmarks/stage_harness.py --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 --stages 0 3 5 $gc > $out/harness_unet$gc.log 2>&1 || { echo "harness unet $gc failed"; tail -20 $out/harness_unet$gc.log; exit 1; }
  cat $out/harness_unet$gc.log
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ops/test_winograd_gpu.py -k "split_patch" > $out/v20_tests.log 2>&1; rc=$?; tail -3 $out/v20_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u benchmarks/wino_variants.py --variants 6 20 --shape 32 128 128 96 --shape 40 128 128 96 --shape 16 128 128 96 --shape 40 64 64 192 --shape 16 64 64 192 --shape 32 64 64 192 --shape 16 128 64 192 --out $out/wino_v20.json > $out/wino_v20.log 2>&1; echo "v20 rc=$?"; cat $out/wino_v20.log
