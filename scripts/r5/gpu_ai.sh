#!/bin/bash
# r5ai: pre-split weights for the split-bf16 implicit GEMMs -- numerics (the whole conv_gemm /
# fused ConvBN GPU file: cfg 7-9 now stage pre-split weights; bit-identity tests), then
# stage-harness A/B (TGPIPE_CG_PRESPLIT_MB=0: in-kernel split) on AmoebaNet n8 stages 5-6,
# n2 stage 1 and ResNet p8 stage 7
export TMPDIR=/tmp
out=gpurun_out/r5ai
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/ops/test_convbn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
for mb in 0 512; do
  export TGPIPE_CG_PRESPLIT_MB=$mb
  h n8_s56_ps$mb --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6
  h n2_s1_ps$mb --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --stages 1
  h resnet_p8_s7_ps$mb --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 7
done
