#!/bin/bash
# r6ay: AmoebaNet's unfused node-sum adds by operation
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6ay
mkdir -p $out
timeout -k 10 300 python -u benchmarks/diag/amoeba_add_probe.py > $out/probe.log 2>&1 || { tail -20 $out/probe.log; exit 1; }
grep -v -i "warn\|amdgpu.ids" $out/probe.log
