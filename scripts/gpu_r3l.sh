# Round 3 call l: reference-balance stage harness (p2/p4/p8) and kernel stats of the
# heaviest stages with the batched-GEMM kernels.
set -o pipefail
out=gpurun_out/r3l
mkdir -p $out
timeout -k 10 300 python benchmarks/stage_harness.py --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 --out $out/stage_p8.json > $out/stage_p8.log 2>&1 || { tail -5 $out/stage_p8.log; exit 1; }
timeout -k 10 300 python benchmarks/stage_harness.py --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --out $out/stage_p4.json > $out/stage_p4.log 2>&1 || { tail -5 $out/stage_p4.log; exit 1; }
timeout -k 10 300 python benchmarks/stage_harness.py --model unet --balance 104 137 --chunks 32 --batch 512 --out $out/stage_p2.json > $out/stage_p2.log 2>&1 || { tail -5 $out/stage_p2.log; exit 1; }
cat $out/stage_p8.log $out/stage_p4.log $out/stage_p2.log | grep stage
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p4s1 -o run -- python3 benchmarks/stage_harness.py --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 1 > $out/p4s1.log 2>&1 || { tail -5 $out/p4s1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p8s3 -o run -- python3 benchmarks/stage_harness.py --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 --stages 3 > $out/p8s3.log 2>&1 || { tail -5 $out/p8s3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p2s0 -o run -- python3 benchmarks/stage_harness.py --model unet --balance 104 137 --chunks 32 --batch 512 --stages 0 > $out/p2s0.log 2>&1 || { tail -5 $out/p2s0.log; exit 1; }
find $out -name '*kernel_trace.csv' -delete
echo DONE
