# Round 3 final check: whole GPU suite, smoke, default bench (U-Net p1 + baseline +
# AmoebaNet n1m32), ResNet-101 p1.
set -o pipefail
out=gpurun_out/r3an
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 5 --warmup 2 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/resnet_kernel_table.py > $out/resnet_table.txt 2> $out/resnet_table.err; echo "resnet rc=$?"; head -1 $out/resnet_table.txt
