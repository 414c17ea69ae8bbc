# End-of-round reference-balance stage runs on the final tree (all three models), for
# profiles/r4/speedup_prediction.md.
set -o pipefail
out=gpurun_out/r4ad
mkdir -p $out
h() {
  local name=$1; shift
  timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/$name.json > $out/$name.log 2>&1 || { echo "$name failed"; tail -20 $out/$name.log; return 1; }
  echo "== $name"; grep '"stage"' $out/$name.log | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['stage'], r['device_ms'], r['host_ms'])"
}
h unet_p2 --model unet --balance 104 137 --chunks 32 --batch 512 --graph-cells || exit 1
h unet_p4 --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --graph-cells || exit 1
h unet_p8 --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 --graph-cells || exit 1
h amoeba_n2m1 --model amoebanet --balance 7 17 --chunks 1 --batch 96 --checkpoint always --graph-cells || exit 1
h amoeba_n2m32 --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --graph-cells || exit 1
h amoeba_n4m32 --model amoebanet --balance 3 6 7 8 --chunks 32 --batch 1152 --graph-cells || exit 1
h amoeba_n8m32 --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --graph-cells || exit 1
h resnet_p2_mb110 --model resnet101 --balance 135 235 --chunks 32 --batch 3520 --checkpoint always --graph-cells --lanes on || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('unet', d['value'], 'base', d['baseline']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'], d['resnet101'].get('baseline',{}).get('value'))"
