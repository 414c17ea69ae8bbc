#!/bin/bash
# r5aw: U-Net stage harness at the reference balances on the final tree (the prediction rows)
export TMPDIR=/tmp
out=gpurun_out/r5aw
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([s['device_ms'] for s in d['stages']])")"; }
h unet_p2 --model unet --balance 104 137 --chunks 32 --batch 512
h unet_p4 --model unet --balance 30 66 84 61 --chunks 16 --batch 512
h unet_p8 --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640
