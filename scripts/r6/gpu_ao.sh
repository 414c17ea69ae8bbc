#!/bin/bash
# r6ao: which aten ops launch ResNet p4 stage 3's library kernels (one micro-batch), then
# the strided Conv-BN choice traces (scripts/r6/gpu_an.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6ao
mkdir -p $out
timeout -k 10 300 python -u benchmarks/diag/op_census.py --lo 260 --hi 370 --batch 22 > $out/census_s3.log 2>&1 || { tail -20 $out/census_s3.log; exit 1; }
grep -v Warning $out/census_s3.log | tail -40
bash scripts/r6/gpu_an.sh
