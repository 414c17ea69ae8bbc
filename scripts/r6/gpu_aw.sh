#!/bin/bash
# r6aw: library / elementwise kernels of AmoebaNet n2m32's stage 1 (layers 9-24, 40 images)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6aw
mkdir -p $out
timeout -k 10 300 python -u benchmarks/diag/op_census.py --model amoebanet --lo 9 --hi 24 --batch 40 > $out/census_amoeba_s1.log 2>&1 || { tail -20 $out/census_amoeba_s1.log; exit 1; }
grep -v -i warn $out/census_amoeba_s1.log | tail -40
