# Round 3 call j: kSub GEMM numerics + sweep; kernel stats of the p4 stage 1 / p1 bench.
set -o pipefail
out=gpurun_out/r3j
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/ops/test_winograd_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $out/tests.log | head -30; exit 1; }
timeout -k 10 600 python -u benchmarks/bg_bench.py --out $out/bg_bench.json > $out/bg_bench.log 2>&1 || { tail -20 $out/bg_bench.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p4s1 -o run -- python3 benchmarks/stage_harness.py --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 1 > $out/p4s1.log 2>&1 || { tail -5 $out/p4s1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p1 -o run -- python3 bench.py --gpus 1 --steps 6 --warmup 2 --sections none > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
find $out -name '*kernel_trace.csv' -delete
echo DONE
