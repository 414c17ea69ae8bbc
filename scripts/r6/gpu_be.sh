#!/bin/bash
# r6be: batched-GEMM Winograd for ResNet's 64 / 128-channel 3x3 layers?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6be
mkdir -p $out
timeout -k 10 300 python -u benchmarks/diag/bg_min_channels_probe.py --out $out/bg_min_channels.json > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
grep shape $out/probe.log
