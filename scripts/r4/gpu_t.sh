# Kernel trace of U-Net p4 stage 1 (the point furthest below the reference curve) with
# captured cells and lanes, as bench.py runs it at N=4.
set -o pipefail
out=gpurun_out/r4t
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_unet_p4_s1 -o run -- python3 benchmarks/stage_harness.py --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 1 --graph-cells --steps 2 > $out/prof_unet_p4_s1.log 2>&1 || { tail -20 $out/prof_unet_p4_s1.log; exit 1; }
grep '"stage"' $out/prof_unet_p4_s1.log
timeout -k 10 300 python -u benchmarks/stage_harness.py --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 1 2 --graph-cells > $out/unet_p4_s12.log 2>&1 || { tail -20 $out/unet_p4_s12.log; exit 1; }
grep '"stage"' $out/unet_p4_s12.log
