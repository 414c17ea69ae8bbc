#!/bin/bash
# r5s: ResNet-101 stage harness at the reference balances after the fitted F(4x4) split-K
# models (ResNet p2 also at the reference's own B=25000, m=1667 sizing)
export TMPDIR=/tmp
out=gpurun_out/r5s
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([s['device_ms'] for s in d['stages']])")"; }
h resnet_p4 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632
h resnet_p8 --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400
h resnet_p2 --model resnet101 --balance 135 235 --chunks 32 --batch 3520 --checkpoint always
h resnet_p2_b25000 --model resnet101 --balance 135 235 --chunks 1667 --batch 25000 --checkpoint always --warmup 1 --steps 1
