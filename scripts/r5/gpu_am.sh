#!/bin/bash
# r5am: the fused small-plane split-K BatchNorm (launch_split_bn_small): fused-op / grouped-op
# / AmoebaNet / ResNet GPU numerics, then the stage harness A/B (TGPIPE_SPLIT_BN=0: split
# reduction + finalize-apply) on AmoebaNet n8 stages 5-6, n2 stage 1, ResNet p8 stage 7
export TMPDIR=/tmp
out=gpurun_out/r5am
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/ops/test_convbn_gpu.py tests/ops/test_group_convbn_gpu.py tests/models -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
for sb in 0 1; do
  export TGPIPE_SPLIT_BN=$sb
  h n8_s56_sb$sb --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6
  h n2_s1_sb$sb --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --stages 1
  h resnet_p8_s7_sb$sb --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 7
done
