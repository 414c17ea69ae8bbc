#!/bin/bash
# r6av: do ResNet's residual joins run fused inside a partition?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6av
mkdir -p $out
timeout -k 10 300 python -u benchmarks/diag/join_probe.py --lo 260 --hi 370 --batch 22 > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
grep tracker $out/probe.log
