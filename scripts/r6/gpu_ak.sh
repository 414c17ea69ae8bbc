#!/bin/bash
# r6ak: split-bf16 batched-GEMM Winograd tile width at ResNet's pipeline micro-batches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6ak
mkdir -p $out
PYTHONPATH=. timeout -k 10 300 python -u benchmarks/diag/bg_tile_probe.py --out $out/bg_tile_probe.json > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
cat $out/probe.log
