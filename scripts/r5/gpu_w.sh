#!/bin/bash
# r5w: host-time breakdown (torch.profiler, all threads) of the launch-bound stages
export TMPDIR=/tmp
out=gpurun_out/r5w
mkdir -p $out
timeout -k 10 600 python -u benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 6 --warmup 2 --steps 1 --torch-profile $out/amoeba_n8 --out $out/h_amoeba.json > $out/amoeba.log 2>&1 || { tail -20 $out/amoeba.log; exit 1; }
timeout -k 10 600 python -u benchmarks/stage_harness.py --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 3 --warmup 2 --steps 1 --torch-profile $out/resnet_p4 --out $out/h_resnet.json > $out/resnet.log 2>&1 || { tail -20 $out/resnet.log; exit 1; }
head -45 $out/amoeba_n8_stage6.txt
head -45 $out/resnet_p4_stage3.txt
