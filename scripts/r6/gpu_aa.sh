#!/bin/bash
# r6aa: ResNet-101 3x3 layers on the fused Winograd kernels instead of the batched-GEMM path
# (TGPIPE_WINOGRAD_BG_MIN_CHANNELS=4096) at the p4 / p8 micro-batches, A/B on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6aa
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
for bg in 4096 256; do
  TGPIPE_WINOGRAD_BG_MIN_CHANNELS=$bg h p4_bg$bg --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 2 3 || exit 1
  TGPIPE_WINOGRAD_BG_MIN_CHANNELS=$bg h p8_bg$bg --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 6 7 || exit 1
done
