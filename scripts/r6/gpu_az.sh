#!/bin/bash
# r6az: the join-mask fallback cleanup: ResNet fused tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6az
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/models/test_resnet_fused_gpu.py tests/ops/test_convbn_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
