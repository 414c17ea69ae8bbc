#!/bin/bash
# r5h: stage harness at the reference balances: AmoebaNet-D(18,256) n2m1 (denominator) /
# n2m32 / n4m32 / n8m32 and ResNet-101 pipeline-2 (config #2) / -4 / -8
export TMPDIR=/tmp
out=gpurun_out/r5h
mkdir -p $out
h() { name=$1; shift; timeout -k 10 900 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name done"; }
h amoeba_n2m1 --model amoebanet --balance 7 17 --chunks 1 --batch 96 --checkpoint always
h amoeba_n2m32 --model amoebanet --balance 9 15 --chunks 32 --batch 1280
h amoeba_n4m32 --model amoebanet --balance 3 6 7 8 --chunks 32 --batch 1152
h amoeba_n8m32 --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280
h resnet_p2 --model resnet101 --balance 135 235 --chunks 32 --batch 3520 --checkpoint always
h resnet_p4 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632
h resnet_p8 --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400
