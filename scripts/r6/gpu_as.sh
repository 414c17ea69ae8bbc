#!/bin/bash
# r6as: the stage harness of every reference experiment again on the final tree (a second box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6as
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/models/test_resnet_fused_gpu.py tests/test_gpu_pipeline.py > $out/tests.log 2>&1 \
  && tail -1 $out/tests.log || { tail -30 $out/tests.log; exit 1; }
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([s['device_ms'] for s in d['stages']])")"; }
h amoeba_n2m1 --model amoebanet --balance 7 17 --chunks 1 --batch 96 --checkpoint always || exit 1
h amoeba_n8m32 --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 || exit 1
h amoeba_n2m32 --model amoebanet --balance 9 15 --chunks 32 --batch 1280 || exit 1
h amoeba_n4m32 --model amoebanet --balance 3 6 7 8 --chunks 32 --batch 1152 || exit 1
h resnet_p4 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 || exit 1
h resnet_p8 --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 || exit 1
h unet_p2 --model unet --balance 104 137 --chunks 32 --batch 512 || exit 1
h unet_p4 --model unet --balance 30 66 84 61 --chunks 16 --batch 512 || exit 1
h unet_p8 --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 || exit 1
h amoeba_n2m32_gc --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --graph-cells || exit 1
h amoeba_n8m32_gc --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --graph-cells || exit 1
h amoeba_n4m32_gc --model amoebanet --balance 3 6 7 8 --chunks 32 --batch 1152 --graph-cells || exit 1
