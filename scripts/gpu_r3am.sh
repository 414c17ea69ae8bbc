# Round 3: ResNet identity gradient accumulated by conv1's backward-data GEMM (GradSink):
# tests, ResNet-101 p1 twice.
set -o pipefail
out=gpurun_out/r3am
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/models/test_resnet_fused_gpu.py tests/ops/test_lib_dgrad_gpu.py tests/ops/test_convbn_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py > $out/resnet_table.txt 2> $out/resnet_table.err; echo "resnet rc=$?"; head -1 $out/resnet_table.txt
PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py > $out/resnet_table2.txt 2> $out/resnet_table2.err; echo "resnet rc=$?"; head -1 $out/resnet_table2.txt
