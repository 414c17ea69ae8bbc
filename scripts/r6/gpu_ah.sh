#!/bin/bash
# r6ah: BatchNorm apply / backward kernels with two 16-byte loads in flight per thread:
# fused-op tests, then stage times new vs previous build interleaved on one box
# (previous build shipped as torchgpipe_amd/_C_old.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6ah
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ops/test_convbn_gpu.py tests/ops/test_group_convbn_gpu.py tests/ops/test_kernels_gpu.py tests/models/test_resnet_fused_gpu.py tests/test_overlap_recompute.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
cp torchgpipe_amd/_C.so /tmp/_C_new.so
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
for rep in 1 2; do
  for v in new old; do
    if [ $v = new ]; then cp /tmp/_C_new.so torchgpipe_amd/_C.so; else cp torchgpipe_amd/_C_old.so torchgpipe_amd/_C.so; fi
    h n1_${v}_$rep --model amoebanet --balance 24 --chunks 32 --batch 1280 || exit 1
    h p4_${v}_$rep --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 3 || exit 1
    h n8_${v}_$rep --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6 || exit 1
  done
done
