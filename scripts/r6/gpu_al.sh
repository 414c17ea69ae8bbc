#!/bin/bash
# r6al: F(4x4) weight-gradient variants at ResNet's pipeline micro-batches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6al
mkdir -p $out
PYTHONPATH=. timeout -k 10 300 python -u benchmarks/diag/wgrad_small_probe.py --out $out/wgrad_small_probe.json > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
grep shape $out/probe.log
