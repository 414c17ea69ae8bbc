# After the stride-2 1x1 fill: the per-shape table with training's cached W^T, and the
# AmoebaNet reference / MI355X-balance stage runs (reduction cells use the fill).
set -o pipefail
out=gpurun_out/r4am
mkdir -p $out
timeout -k 10 600 python -u benchmarks/convbn_bench.py --micro-batch 40 --out $out/convbn_bench_n40_wt.json > $out/convbn.log 2>&1 || { tail -20 $out/convbn.log; exit 1; }
tail -1 $out/convbn.log
h() {
  local name=$1; shift
  timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/$name.json > $out/$name.log 2>&1 || { echo "$name failed"; tail -20 $out/$name.log; return 1; }
  echo "== $name"; grep '"stage"' $out/$name.log | python -c "
import json,sys
print([r['device_ms'] for r in map(json.loads, sys.stdin)])"
}
h amoeba_n2m1 --model amoebanet --balance 7 17 --chunks 1 --batch 96 --checkpoint always --graph-cells || exit 1
h amoeba_n2m32 --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --graph-cells || exit 1
h amoeba_n4m32 --model amoebanet --balance 3 6 7 8 --chunks 32 --batch 1152 --graph-cells || exit 1
h amoeba_n8m32 --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --graph-cells || exit 1
h amoeba_n2m32_tuned --model amoebanet --balance 11 13 --chunks 32 --batch 1280 --graph-cells || exit 1
h amoeba_n4m32_tuned --model amoebanet --balance 5 6 6 7 --chunks 32 --batch 1152 --graph-cells || exit 1
h amoeba_n8m32_tuned --model amoebanet --balance 2 3 3 3 3 3 3 4 --chunks 32 --batch 1280 --graph-cells || exit 1
