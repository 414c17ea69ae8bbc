#!/bin/bash
# r5p: stage harness of the current tuned balances vs the transfer-aware searched ones
# (scripts/r5/tune_transfer.py at 100 GB/s)
export TMPDIR=/tmp
out=gpurun_out/r5p
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([s['device_ms'] for s in d['stages']])")"; }
h unet_p4_tuned --model unet --balance 38 55 74 74 --chunks 16 --batch 512
h unet_p4_search --model unet --balance 39 55 76 71 --chunks 16 --batch 512
h unet_p8_tuned --model unet --balance 18 26 27 30 22 44 40 34 --chunks 40 --batch 640
h unet_p8_search --model unet --balance 20 23 28 30 25 40 44 31 --chunks 40 --batch 640
h amoeba_n2m32_tuned --model amoebanet --balance 11 13 --chunks 32 --batch 1280
h amoeba_n2m32_search --model amoebanet --balance 10 14 --chunks 32 --batch 1280
h amoeba_n8m32_tuned --model amoebanet --balance 2 3 3 3 3 3 3 4 --chunks 32 --batch 1280
h amoeba_n8m32_search --model amoebanet --balance 2 2 3 3 3 3 3 5 --chunks 32 --batch 1280
h amoeba_n4m32_tuned --model amoebanet --balance 5 6 6 7 --chunks 32 --batch 1152
