# Round 3 call i: kernel stats of p4 stage 1 / p8 stage 3 and of the p1 bench after the
# batched-GEMM dispatch.
set -o pipefail
out=gpurun_out/r3i
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p4s1 -o run -- python3 benchmarks/stage_harness.py --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 1 > $out/p4s1.log 2>&1 || { tail -5 $out/p4s1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p8s3 -o run -- python3 benchmarks/stage_harness.py --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 --stages 3 > $out/p8s3.log 2>&1 || { tail -5 $out/p8s3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p1 -o run -- python3 bench.py --gpus 1 --steps 6 --warmup 2 --sections none > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
find $out -name '*kernel_trace.csv' -delete
echo DONE
