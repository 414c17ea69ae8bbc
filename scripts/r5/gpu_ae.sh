#!/bin/bash
# r5ae: split-bf16 weight gradient in the model path: numerics, then U-Net p1 headline A/B
# (TGPIPE_WGRAD_EMU=0 / 1, alternating on one box) and the U-Net p8 deep stages
export TMPDIR=/tmp
out=gpurun_out/r5ae
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/ops/test_winograd_gpu.py -x -q --timeout 120 --timeout-method thread -k "module_weight_gradient or f4_wgrad" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for i in 1 2; do
  for e in 0 1; do
    TGPIPE_WGRAD_EMU=$e timeout -k 10 300 python -u bench.py --sections none --steps 8 > $out/bench_emu${e}_$i.json 2> $out/bench_emu${e}_$i.log || { tail -20 $out/bench_emu${e}_$i.log; exit 1; }
    echo "emu=$e run $i: $(python -c "import json;print(json.load(open('$out/bench_emu${e}_$i.json'))['value'])")"
  done
done
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([s['device_ms'] for s in d['stages']])")"; }
h unet_p8 --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640
h unet_p4 --model unet --balance 30 66 84 61 --chunks 16 --batch 512
