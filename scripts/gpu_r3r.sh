# Round 3: per-stage device times of U-Net p2/p4/p8 at the reference balances with the
# current kernels (batched-GEMM Winograd for >= 256 channels), for the speed-up prediction.
set -o pipefail
out=gpurun_out/r3r
mkdir -p $out
timeout -k 10 300 python benchmarks/stage_harness.py --balance 104 137 --chunks 32 --batch 512 --out $out/harness_p2_ref.json > $out/p2.log 2>&1 || { tail -20 $out/p2.log; exit 1; }
timeout -k 10 300 python benchmarks/stage_harness.py --balance 30 66 84 61 --chunks 16 --batch 512 --out $out/harness_p4_ref.json > $out/p4.log 2>&1 || { tail -20 $out/p4.log; exit 1; }
timeout -k 10 300 python benchmarks/stage_harness.py --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 --out $out/harness_p8_ref.json > $out/p8.log 2>&1 || { tail -20 $out/p8.log; exit 1; }
cat $out/p2.log $out/p4.log $out/p8.log | grep stage
