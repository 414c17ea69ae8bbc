# Batched-GEMM Winograd from 128 / 64 channels (TGPIPE_WINOGRAD_BG_MIN_CHANNELS) vs the
# shipped 256: U-Net p4 stages 1-2 and p2 / p8 slowest stages, U-Net p1 bench.
set -o pipefail
out=gpurun_out/r4ap
mkdir -p $out
h() {
  local name=$1; shift
  timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/$name.json > $out/$name.log 2>&1 || { echo "$name failed"; tail -20 $out/$name.log; return 1; }
  echo "== $name"; grep '"stage"' $out/$name.log | python -c "
import json,sys
print([r['device_ms'] for r in map(json.loads, sys.stdin)])"
}
for bgmin in 256 128 64; do
  export TGPIPE_WINOGRAD_BG_MIN_CHANNELS=$bgmin
  h unet_p4_bg$bgmin --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 1 2 --graph-cells || exit 1
  h unet_p8_bg$bgmin --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 --stages 1 3 5 --graph-cells || exit 1
  timeout -k 10 600 python -u bench.py --sections none > $out/bench_bg$bgmin.log 2>&1 || { tail -20 $out/bench_bg$bgmin.log; exit 1; }
  echo "bench bg$bgmin $(tail -1 $out/bench_bg$bgmin.log | cut -c1-130)"
done
