# Round 3: library backward-data for the fused ReLU-Conv-BN ops (per-geometry timed choice):
# tests, AmoebaNet n1m32 A/B (TGPIPE_LIB_DGRAD=0), ResNet-101 p1, ResNet strided-conv probe.
set -o pipefail
out=gpurun_out/r3ag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/ops/test_lib_dgrad_gpu.py tests/ops/test_convbn_gpu.py tests/ops/test_group_convbn_gpu.py tests/models/test_resnet_fused_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 400 python bench.py --model amoebanet --steps 5 --warmup 2 --sections none > $out/amoeba_lib.json 2> $out/amoeba_lib.err || { tail -20 $out/amoeba_lib.err; exit 1; }
cat $out/amoeba_lib.json
TGPIPE_LIB_DGRAD=0 timeout -k 10 400 python bench.py --model amoebanet --steps 5 --warmup 2 --sections none > $out/amoeba_nolib.json 2> $out/amoeba_nolib.err || { tail -20 $out/amoeba_nolib.err; exit 1; }
cat $out/amoeba_nolib.json
timeout -k 10 400 python bench.py --model amoebanet --steps 5 --warmup 2 --sections none > $out/amoeba_lib2.json 2> $out/amoeba_lib2.err || { tail -20 $out/amoeba_lib2.err; exit 1; }
cat $out/amoeba_lib2.json
PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py > $out/resnet_table.txt 2> $out/resnet_table.err; echo "resnet rc=$?"; head -1 $out/resnet_table.txt
PYTHONPATH=. timeout -k 10 200 python benchmarks/diag/resnet_strided_probe.py > $out/strided_probe.jsonl 2> $out/strided_probe.err; echo "probe rc=$?"; cat $out/strided_probe.jsonl
