#!/bin/bash
# r6bp: caching-allocator device allocations per steady-state step (ResNet p1, U-Net p1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6bp
mkdir -p $out
timeout -k 10 300 python -u benchmarks/diag/alloc_probe.py --model resnet > $out/resnet.log 2>&1 || { tail -20 $out/resnet.log; exit 1; }
grep step $out/resnet.log
timeout -k 10 300 python -u benchmarks/diag/alloc_probe.py --model unet > $out/unet.log 2>&1 || { tail -20 $out/unet.log; exit 1; }
grep step $out/unet.log
