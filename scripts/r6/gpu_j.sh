#!/bin/bash
# r6j: the BatchNorm gradient-accumulation A/B (gpu_i.sh), then the first two memory rows
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/r6/gpu_i.sh || exit 1
export TMPDIR=/tmp
out=gpurun_out/r6e
mkdir -p $out
run() { tag=$1; shift; timeout -k 10 ${LIMIT:-560} python -u benchmarks/memory.py "$@" --out $out/$tag.json > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; exit 1; }; tail -1 $out/$tag.log | cut -c1-400; }
run amoebanet_72_512_p8 amoebanet --experiment pipeline-8 || exit 1
run unet_48_160_p8 unet --experiment pipeline-8
