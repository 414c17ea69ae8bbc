# Round 3: fused 3x3 Conv-BN-ReLU x.grad accuracy diagnosis; the ResNet-101 kernel trace.
set -o pipefail
out=gpurun_out/r3y
mkdir -p $out
PYTHONPATH=. timeout -k 10 200 python benchmarks/diag/resnet_fused_diag2.py 2>&1 | grep -v amdgpu.ids | tee $out/diag2.log
PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py > $out/resnet_fused_table.txt 2> $out/resnet_fused_table.err; echo "fused rc=$?"; head -3 $out/resnet_fused_table.txt
PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py --plain > $out/resnet_plain_table.txt 2> $out/resnet_plain_table.err; echo "plain rc=$?"; head -3 $out/resnet_plain_table.txt
exit 0
