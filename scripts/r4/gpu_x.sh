# One-tile GEMM waves alternate two accumulators (forward / weight gradient): numerics,
# mb-40 sweep, AmoebaNet n8m32 stage 6 and n2m1.
set -o pipefail
out=gpurun_out/r4x
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/ops/test_convbn_gpu.py tests/ops/test_group_convbn_gpu.py -q -x --timeout 120 --timeout-method thread -k "not avgpool" > $out/conv_tests.log 2>&1 || { tail -30 $out/conv_tests.log; exit 1; }
tail -2 $out/conv_tests.log
timeout -k 10 300 python -u benchmarks/convgemm_sweep.py --micro-batch 40 --out $out/convgemm_sweep_n40.json > $out/sweep.log 2>&1 || { tail -20 $out/sweep.log; exit 1; }
timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 6 --graph-cells > $out/harness_s6.log 2>&1 || { tail -20 $out/harness_s6.log; exit 1; }
grep '"stage"' $out/harness_s6.log
timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 7 17 --chunks 1 --batch 96 --checkpoint always --graph-cells > $out/n2m1.log 2>&1 || { tail -20 $out/n2m1.log; exit 1; }
grep '"stage"' $out/n2m1.log
