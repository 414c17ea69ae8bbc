#!/bin/bash
# r6k: the fused split BatchNorm widened to 14^2 planes -- its fp64 tests, then an A/B
# against the round-5 limit (TGPIPE_SPLIT_BN=64) on the stages it touches, then the
# single-GPU memory maximum U-Net(24,300)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6k
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ops/test_convbn_gpu.py tests/ops/test_group_convbn_gpu.py -k "split_small or fused_split or group" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
for sb in 256 64; do
  TGPIPE_SPLIT_BN=$sb h p4s3_sb$sb --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 2 3 || exit 1
  TGPIPE_SPLIT_BN=$sb h p8s7_sb$sb --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 6 7 || exit 1
  TGPIPE_SPLIT_BN=$sb h n8_sb$sb --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 3 5 || exit 1
  TGPIPE_SPLIT_BN=$sb h n2_sb$sb --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --stages 1 || exit 1
done
timeout -k 10 560 python -u benchmarks/memory.py unet -B 24 -C 300 --balance 1077 --chunks 32 --out gpurun_out/r6e/unet_24_300_p1.json > gpurun_out/r6e/unet_24_300_p1.log 2>&1 || { tail -5 gpurun_out/r6e/unet_24_300_p1.log; exit 1; }
tail -1 gpurun_out/r6e/unet_24_300_p1.log | cut -c1-300
