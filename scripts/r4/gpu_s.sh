# AmoebaNet n8m32 stage 6 with the forward / backward-data split-K capped (TGPIPE_CG_SPLIT_CAP)
# and the n2m1 denominator's two stages on the current kernels.
set -o pipefail
out=gpurun_out/r4s
mkdir -p $out
for cap in 0 1 2; do
  TGPIPE_CG_SPLIT_CAP=$cap timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 6 --graph-cells > $out/s6_cap$cap.log 2>&1 || { tail -20 $out/s6_cap$cap.log; exit 1; }
  echo "cap $cap: $(grep '"stage"' $out/s6_cap$cap.log)"
done
TGPIPE_CG_SPLIT_CAP=1 timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 --graph-cells > $out/s5_cap1.log 2>&1 || { tail -20 $out/s5_cap1.log; exit 1; }
echo "s5 cap 1: $(grep '"stage"' $out/s5_cap1.log)"
timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 7 17 --chunks 1 --batch 96 --checkpoint always --graph-cells --out $out/amoeba_n2m1.json > $out/n2m1.log 2>&1 || { tail -20 $out/n2m1.log; exit 1; }
grep '"stage"' $out/n2m1.log
