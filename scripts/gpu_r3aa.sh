# Round 3: full default bench (U-Net p1 headline + no-GPipe baseline + AmoebaNet n1m32),
# fused ResNet-101 p1 with strided convolutions on MIOpen, AmoebaNet kernel trace (eager).
set -o pipefail
out=gpurun_out/r3aa
mkdir -p $out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/models/test_resnet_fused_gpu.py > $out/tests.log 2>&1; rc=$?
tail -2 $out/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 5 --warmup 2 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py > $out/resnet_fused_table.txt 2> $out/resnet_fused_table.err; echo "fused rc=$?"; head -1 $out/resnet_fused_table.txt
bash scripts/profile_bench.sh amoeba_r3aa --model amoebanet --graph off --steps 3 --warmup 2 --sections none || exit 1
head -32 gpurun_out/prof_amoeba_r3aa/summary.md
