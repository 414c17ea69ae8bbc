# Reference-balance stage predictions with the round-4 engine (captured cells, lanes as in
# bench.py): every stage of U-Net p2/p4/p8, AmoebaNet n2m32/n4m32/n8m32 and the n2m1
# denominator, ResNet-101 pipeline-2 (chunks 32, always).
set -o pipefail
out=gpurun_out/r4h
mkdir -p $out
h() {  # name, args...
  local name=$1; shift
  timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/$name.json > $out/$name.log 2>&1 || { echo "$name failed"; tail -20 $out/$name.log; return 1; }
  echo "== $name"; grep '"stage"' $out/$name.log | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['stage'], r['device_ms'], r['host_ms'], r.get('graph_launch_ms'), r['peak_mem_gib'])"
}
h unet_p2 --model unet --balance 104 137 --chunks 32 --batch 512 --graph-cells || exit 1
h unet_p4 --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --graph-cells || exit 1
h unet_p8 --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 --graph-cells || exit 1
h amoeba_n2m1 --model amoebanet --balance 7 17 --chunks 1 --batch 96 --checkpoint always --graph-cells || exit 1
h amoeba_n2m32 --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --graph-cells || exit 1
h amoeba_n4m32 --model amoebanet --balance 3 6 7 8 --chunks 32 --batch 1152 --graph-cells || exit 1
h amoeba_n8m32 --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --graph-cells || exit 1
h resnet_p2 --model resnet101 --balance 135 235 --chunks 32 --batch 480 --checkpoint always --graph-cells || exit 1
