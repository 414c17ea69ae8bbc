# Round 3 call b: in-kernel gradient accumulation tests, kernel stats of the heaviest
# reference-balance stages (p8 stage 3, p4 stage 2), default bench.
set -o pipefail
out=gpurun_out/r3b
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gradacc.py tests/test_overlap_recompute.py tests/ops/test_winograd_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $out/tests.log | head -30; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p8s3 -o run -- python3 benchmarks/stage_harness.py --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 --stages 3 > $out/p8s3.log 2>&1 || { tail -5 $out/p8s3.log; exit 1; }
tail -1 $out/p8s3.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p4s2 -o run -- python3 benchmarks/stage_harness.py --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 2 > $out/p4s2.log 2>&1 || { tail -5 $out/p4s2.log; exit 1; }
tail -1 $out/p4s2.log
find $out -name '*.db' -delete
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --sections none > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cut -c1-300 $out/bench.json
grep -c "AccumulateGrad" $out/bench.err || true
