# Batched stride-phase backward-data: numerics of every strided geometry, then the
# mb-40 per-shape table (3x3 stride-2 rows against MIOpen) and the ResNet strided probe.
set -o pipefail
out=gpurun_out/r4ac
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/ops/test_convbn_gpu.py tests/ops/test_lib_dgrad_gpu.py -q -x --timeout 120 --timeout-method thread -k "conv_gemm_matches or phases or lib_dgrad" > $out/conv_tests.log 2>&1 || { tail -30 $out/conv_tests.log; exit 1; }
tail -2 $out/conv_tests.log
timeout -k 10 300 python -u benchmarks/convbn_bench.py --micro-batch 40 --out $out/convbn_bench_n40.json > $out/convbn_bench.log 2>&1 || { tail -20 $out/convbn_bench.log; exit 1; }
tail -1 $out/convbn_bench.log
timeout -k 10 300 python -u benchmarks/diag/resnet_strided_probe.py > $out/resnet_strided_probe.jsonl 2> $out/resnet_strided_probe.err || { tail -20 $out/resnet_strided_probe.err; exit 1; }
