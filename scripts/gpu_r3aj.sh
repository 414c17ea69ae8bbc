# Round 3: AmoebaNet-D(18,256) reference-balance stage times (one GPU per stage, eager,
# three-stream cells as bench.py runs them) for the n2m1 / n2m32 / n4m32 / n8m32 speed-up
# prediction over the reference's n2m1 denominator.
set -o pipefail
out=gpurun_out/r3aj
mkdir -p $out
H="timeout -k 10 400 python benchmarks/stage_harness.py --model amoebanet --cell-streams 3"
$H --balance 7 17 --chunks 1 --batch 96 --checkpoint always --out $out/amoeba_n2m1.json > $out/n2m1.log 2>&1 || { tail -20 $out/n2m1.log; exit 1; }
grep stage $out/n2m1.log
$H --balance 9 15 --chunks 32 --batch 1280 --out $out/amoeba_n2m32.json > $out/n2m32.log 2>&1 || { tail -20 $out/n2m32.log; exit 1; }
grep stage $out/n2m32.log
$H --balance 3 6 7 8 --chunks 32 --batch 1152 --out $out/amoeba_n4m32.json > $out/n4m32.log 2>&1 || { tail -20 $out/n4m32.log; exit 1; }
grep stage $out/n4m32.log
$H --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --out $out/amoeba_n8m32.json > $out/n8m32.log 2>&1 || { tail -20 $out/n8m32.log; exit 1; }
grep stage $out/n8m32.log
