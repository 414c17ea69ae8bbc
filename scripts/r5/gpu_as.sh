#!/bin/bash
# r5as: memory benchmark rows on the latest tree (pre-split weights off in the memory-lean mode,
# released as each micro-batch's backward runs): AmoebaNet-D(72,512) p8, U-Net(48,160) p8
export TMPDIR=/tmp
out=gpurun_out/r5as
mkdir -p $out
run() { tag=$1; shift; timeout -k 10 560 python -u benchmarks/memory.py "$@" --out $out/$tag.json > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; exit 1; }; tail -1 $out/$tag.log | cut -c1-400; }
run amoebanet_72_512_p8 amoebanet --experiment pipeline-8
run unet_48_160_p8 unet --experiment pipeline-8
