#!/bin/bash
# r5l: where the host time of the launch-bound stages goes: cProfile of the stage harness
# (eager, 1 timed step) for ResNet p4 stage 2 (m=256, 22 images) and AmoebaNet n8m32 stage 6
export TMPDIR=/tmp
out=gpurun_out/r5l
mkdir -p $out
timeout -k 10 600 python -u -m cProfile -o $out/resnet_p4_s2.prof benchmarks/stage_harness.py --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 2 --warmup 2 --steps 1 > $out/resnet.log 2>&1 || { tail -20 $out/resnet.log; exit 1; }
timeout -k 10 600 python -u -m cProfile -o $out/amoeba_n8_s6.prof benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 6 --warmup 2 --steps 1 > $out/amoeba.log 2>&1 || { tail -20 $out/amoeba.log; exit 1; }
grep '"stage"' $out/*.log | cut -c1-200
