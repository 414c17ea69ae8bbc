#!/bin/bash
# r6m: the 8-GPU memory maximum U-Net(48,576) pipeline-8 on this round's tree, stage by stage
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6e
timeout -k 10 1100 python -u benchmarks/memory.py unet -B 48 -C 576 --balance 852 123 32 32 35 33 35 991 --chunks 128 --out gpurun_out/r6e/unet_48_576_p8.json > gpurun_out/r6e/unet_48_576_p8.log 2>&1 || { tail -5 gpurun_out/r6e/unet_48_576_p8.log; exit 1; }
tail -1 gpurun_out/r6e/unet_48_576_p8.log | cut -c1-300
