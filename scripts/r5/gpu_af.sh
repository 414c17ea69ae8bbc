#!/bin/bash
# r5af: host-time breakdown of AmoebaNet n2m32 stage 1 (the last, 15-layer stage) and of
# ResNet p8 stage 7, after the host trims
export TMPDIR=/tmp
out=gpurun_out/r5af
mkdir -p $out
timeout -k 10 600 python -u benchmarks/stage_harness.py --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --stages 1 --warmup 2 --steps 1 --torch-profile $out/amoeba_n2 --out $out/h_amoeba.json > $out/amoeba.log 2>&1 || { tail -20 $out/amoeba.log; exit 1; }
head -40 $out/amoeba_n2_stage1.txt
