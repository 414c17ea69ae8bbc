#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6p
timeout -k 10 400 python -u scripts/debug/resnet_determinism.py deterministic > gpurun_out/r6p/determinism.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r6p/determinism.log | tail -40
exit $rc
