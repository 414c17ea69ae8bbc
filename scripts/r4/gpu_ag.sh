# AmoebaNet MI355X balances measured as whole stages on the final tree (bench.py `tuned`).
set -o pipefail
out=gpurun_out/r4ag
mkdir -p $out
h() {
  local name=$1; shift
  timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/$name.json > $out/$name.log 2>&1 || { echo "$name failed"; tail -20 $out/$name.log; return 1; }
  echo "== $name"; grep '"stage"' $out/$name.log | python -c "
import json,sys
print([r['device_ms'] for r in map(json.loads, sys.stdin)])"
}
h amoeba_n2m32_tuned --model amoebanet --balance 11 13 --chunks 32 --batch 1280 --graph-cells || exit 1
h amoeba_n4m32_tuned --model amoebanet --balance 5 6 6 7 --chunks 32 --batch 1152 --graph-cells || exit 1
h amoeba_n8m32_tuned --model amoebanet --balance 2 3 3 3 3 3 3 4 --chunks 32 --batch 1280 --graph-cells || exit 1
h amoeba_n8m32_tuned2 --model amoebanet --balance 3 3 2 3 3 3 3 4 --chunks 32 --batch 1280 --graph-cells || exit 1
