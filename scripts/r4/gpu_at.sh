# U-Net MI355X balances (bench.py `tuned` at N > 1) as whole stages on the final tree.
set -o pipefail
out=gpurun_out/r4at
mkdir -p $out
h() {
  local name=$1; shift
  timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/$name.json > $out/$name.log 2>&1 || { echo "$name failed"; tail -20 $out/$name.log; return 1; }
  echo "== $name"; grep '"stage"' $out/$name.log | python -c "
import json,sys
print([r['device_ms'] for r in map(json.loads, sys.stdin)])"
}
h unet_p2_tuned --model unet --balance 100 141 --chunks 32 --batch 512 --graph-cells || exit 1
h unet_p4_tuned --model unet --balance 44 53 70 74 --chunks 16 --batch 512 --graph-cells || exit 1
h unet_p8_tuned --model unet --balance 18 21 29 29 26 41 44 33 --chunks 40 --batch 640 --graph-cells || exit 1
timeout -k 10 600 python -u bench.py --sections baseline > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('p1', d['value'], 'baseline', d['baseline']['value'])"
