#!/bin/bash
# r5g: stage harness at the reference balances (U-Net p2/p4/p8), and bench.py N=1 (U-Net
# p1 + no-GPipe baseline + AmoebaNet n1m32 + ResNet p1 + ResNet baseline) on this tree
export TMPDIR=/tmp
out=gpurun_out/r5g
mkdir -p $out
timeout -k 10 500 python -u bench.py > $out/bench_n1.json 2> $out/bench_n1.log || { echo "bench failed"; tail -20 $out/bench_n1.log; exit 1; }
python -c "import json;d=json.load(open('$out/bench_n1.json'));print('unet',d['value'],'baseline',d['baseline']['value'],'amoeba',d['amoebanet']['value'],'resnet',d['resnet101']['value'],d['resnet101']['baseline']['value'])"
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name done"; }
h unet_p2 --model unet --balance 104 137 --chunks 32 --batch 512
h unet_p4 --model unet --balance 30 66 84 61 --chunks 16 --batch 512
h unet_p8 --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640
