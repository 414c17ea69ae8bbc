# Round 3: stage times of the MI355X (tuned) U-Net balances, to check the interpolated
# prediction (profiles/r3/speedup_prediction.md).
set -o pipefail
out=gpurun_out/r3ap
mkdir -p $out
timeout -k 10 300 python benchmarks/stage_harness.py --balance 44 53 70 74 --chunks 16 --batch 512 --out $out/harness_p4_tuned.json > $out/p4.log 2>&1 || { tail -20 $out/p4.log; exit 1; }
grep stage $out/p4.log
timeout -k 10 300 python benchmarks/stage_harness.py --balance 18 21 29 29 26 41 44 33 --chunks 40 --batch 640 --out $out/harness_p8_tuned.json > $out/p8.log 2>&1 || { tail -20 $out/p8.log; exit 1; }
grep stage $out/p8.log
timeout -k 10 300 python benchmarks/stage_harness.py --balance 100 141 --chunks 32 --batch 512 --out $out/harness_p2_tuned.json > $out/p2.log 2>&1 || { tail -20 $out/p2.log; exit 1; }
grep stage $out/p2.log
