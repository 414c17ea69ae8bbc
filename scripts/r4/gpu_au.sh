# Re-derived U-Net MI355X balances (scripts/balance_from_harness.py over the final-tree
# reference + tuned stage runs) measured as whole stages.
set -o pipefail
out=gpurun_out/r4au
mkdir -p $out
h() {
  local name=$1; shift
  timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/$name.json > $out/$name.log 2>&1 || { echo "$name failed"; tail -20 $out/$name.log; return 1; }
  echo "== $name"; grep '"stage"' $out/$name.log | python -c "
import json,sys
print([r['device_ms'] for r in map(json.loads, sys.stdin)])"
}
h unet_p4_tuned2 --model unet --balance 38 55 74 74 --chunks 16 --batch 512 --graph-cells || exit 1
h unet_p8_tuned2 --model unet --balance 18 26 27 30 22 44 40 34 --chunks 40 --batch 640 --graph-cells || exit 1
