# Round 3: timed strided Conv-BN path choice for ResNet (fused implicit GEMM vs MIOpen + BN):
# tests, ResNet-101 p1 twice; rocprofv3 kernel trace of the U-Net p1 headline (final tree).
set -o pipefail
out=gpurun_out/r3aq
mkdir -p $out
TGPIPE_STRIDED_CHOICE=1 timeout -k 10 600 python -u -m pytest tests/models/test_resnet_fused_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
TGPIPE_STRIDED_CHOICE=1 PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py > $out/resnet_table.txt 2> $out/resnet_table.err; echo "resnet rc=$?"; head -1 $out/resnet_table.txt
TGPIPE_STRIDED_CHOICE=0 PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py > $out/resnet_table_off.txt 2> $out/resnet_table_off.err; echo "resnet off rc=$?"; head -1 $out/resnet_table_off.txt
TGPIPE_STRIDED_CHOICE=1 PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py > $out/resnet_table2.txt 2> $out/resnet_table2.err; echo "resnet rc=$?"; head -1 $out/resnet_table2.txt
bash scripts/profile_bench.sh unet_p1_r3 --steps 5 --warmup 2 --sections none || exit 1
head -30 gpurun_out/prof_unet_p1_r3/summary.md
