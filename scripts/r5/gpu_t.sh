#!/bin/bash
# r5t: ResNet p2 at the reference's B=25000 / m=1667 (uneven micro-batches), U-Net stage
# harness after the F(4x4) split-K models, batched-GEMM tile/split sweep
export TMPDIR=/tmp
out=gpurun_out/r5t
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([s['device_ms'] for s in d['stages']])")"; }
h resnet_p2_b25000 --model resnet101 --balance 135 235 --chunks 1667 --batch 25000 --checkpoint always --warmup 1 --steps 1
h unet_p2 --model unet --balance 104 137 --chunks 32 --batch 512
h unet_p4 --model unet --balance 30 66 84 61 --chunks 16 --batch 512
h unet_p8 --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640
h unet_p4_tuned --model unet --balance 38 55 74 74 --chunks 16 --batch 512
h unet_p8_tuned --model unet --balance 18 26 27 30 22 44 40 34 --chunks 40 --batch 640
timeout -k 10 300 python -u benchmarks/split_sweep.py --ops bg --out $out/bg_sweep.json > $out/bg_sweep.log 2>&1 || { tail -20 $out/bg_sweep.log; exit 1; }
echo done
