#!/bin/bash
# r5av: AmoebaNet / ResNet stage harness at the reference balances on the final tree (pre-split,
# fused small-plane split BatchNorm, re-timed plan tables): the prediction rows
export TMPDIR=/tmp
out=gpurun_out/r5av
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([s['device_ms'] for s in d['stages']])")"; }
h amoeba_n8m32 --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280
h amoeba_n2m32 --model amoebanet --balance 9 15 --chunks 32 --batch 1280
h amoeba_n4m32 --model amoebanet --balance 3 6 7 8 --chunks 32 --batch 1152
h amoeba_n2m1 --model amoebanet --balance 7 17 --chunks 1 --batch 96 --checkpoint always
h resnet_p4 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632
h resnet_p8 --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400
