#!/bin/bash
# r6aq: strided Conv-BN picks per micro-batch size
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6aq
mkdir -p $out
timeout -k 10 400 python -u benchmarks/diag/strided_picks.py --batches 15 22 36 110 --out $out/strided_picks.json > $out/picks.log 2>&1 || { tail -20 $out/picks.log; exit 1; }
grep batch $out/picks.log
