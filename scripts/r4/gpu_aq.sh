# Fused F(4x4) variant per stage (TGPIPE_F4_FUSED_VARIANT; shipped 6): U-Net p4 stage 1 and
# the U-Net p1 bench headline.
set -o pipefail
out=gpurun_out/r4aq
mkdir -p $out
for v in 6 7 12 18 14; do
  export TGPIPE_F4_FUSED_VARIANT=$v
  timeout -k 10 600 python -u benchmarks/stage_harness.py --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 1 --graph-cells --out $out/unet_p4_s1_v$v.json > $out/unet_p4_s1_v$v.log 2>&1 || { tail -20 $out/unet_p4_s1_v$v.log; exit 1; }
  timeout -k 10 600 python -u bench.py --sections none > $out/bench_v$v.log 2>&1 || { tail -20 $out/bench_v$v.log; exit 1; }
  echo "v$v stage1 $(grep '"stage"' $out/unet_p4_s1_v$v.log | python -c 'import json,sys;print([json.loads(l)["device_ms"] for l in sys.stdin])') p1 $(tail -1 $out/bench_v$v.log | python -c 'import json,sys;print(json.loads(sys.stdin.read())["value"])')"
done
