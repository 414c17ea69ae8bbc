# Whole GPU suite on the current tree, then every reference-balance AmoebaNet stage
# (n2m1 / n2m32 / n4m32 / n8m32) with the round-4 kernels and tables, and the default bench.
set -o pipefail
out=gpurun_out/r4u
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || { grep -B5 -A30 "^E  \|Error" $out/gpu_tests.log | head -60; exit 1; }
h() {
  local name=$1; shift
  timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/$name.json > $out/$name.log 2>&1 || { echo "$name failed"; tail -20 $out/$name.log; return 1; }
  echo "== $name"; grep '"stage"' $out/$name.log | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['stage'], r['device_ms'], r['host_ms'])"
}
h amoeba_n2m1 --model amoebanet --balance 7 17 --chunks 1 --batch 96 --checkpoint always --graph-cells || exit 1
h amoeba_n2m32 --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --graph-cells || exit 1
h amoeba_n4m32 --model amoebanet --balance 3 6 7 8 --chunks 32 --batch 1152 --graph-cells || exit 1
h amoeba_n8m32 --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --graph-cells || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('unet', d['value'], 'base', d['baseline']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'], d['resnet101'].get('baseline',{}).get('value'))"
