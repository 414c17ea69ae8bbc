# Round 3: (1) AmoebaNet-D(18,256) per-layer stage times at micro-batch 40 (32 micro-batches,
# three-stream cells) for MI355X balances; (2) ResNet residual join as one op (conv3 + bn3 +
# identity add + ReLU): tests and ResNet-101 p1.
set -o pipefail
out=gpurun_out/r3ak
mkdir -p $out
timeout -k 10 600 python benchmarks/stage_harness.py --model amoebanet --cell-streams 3 --balance 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 --chunks 32 --batch 1280 --out $out/amoeba_layers_mb40.json > $out/layers.log 2>&1 || { tail -20 $out/layers.log; exit 1; }
grep -c stage $out/layers.log
timeout -k 10 600 python -u -m pytest tests/models/test_resnet_fused_gpu.py tests/models/test_resnet_fusion_cpu.py tests/ops/test_lib_dgrad_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py > $out/resnet_table.txt 2> $out/resnet_table.err; echo "resnet rc=$?"; head -1 $out/resnet_table.txt
PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py --rows 60 > $out/resnet_table2.txt 2> $out/resnet_table2.err; echo "resnet rc=$?"; head -1 $out/resnet_table2.txt
