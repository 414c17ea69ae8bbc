#!/bin/bash
# r6e: the memory maxima on this round's tree (benchmarks/memory.py, stage by stage, with
# the per-stage breakdown): AmoebaNet-D(72,512) p8, U-Net(48,160) p8, U-Net(24,300) p1,
# U-Net(48,576) p8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6e
mkdir -p $out
run() { tag=$1; shift; timeout -k 10 ${LIMIT:-560} python -u benchmarks/memory.py "$@" --out $out/$tag.json > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; exit 1; }; tail -1 $out/$tag.log | cut -c1-400; }
run amoebanet_72_512_p8 amoebanet --experiment pipeline-8
run unet_48_160_p8 unet --experiment pipeline-8
run unet_24_300_p1 unet -B 24 -C 300 --balance 1077 --chunks 32
LIMIT=900 run unet_48_576_p8 unet -B 48 -C 576 --balance 852 123 32 32 35 33 35 991 --chunks 128
