#!/bin/bash
# r5v: does issuing the backward from a helper thread lift the launch-bound stages?
# (AmoebaNet n8m32 stages 5/6, n2m32 stage 1; ResNet p4 stage 3, p8 stage 7), plus the
# shared-GPU rehearsal of the option
export TMPDIR=/tmp
out=gpurun_out/r5v
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
timeout -k 10 400 python -u -m pytest tests/distributed/test_shared_gpu_rehearsal.py -x -q --timeout 200 \
  --timeout-method thread -k "backward_thread" > $out/rehearsal.log 2>&1 || { tail -30 $out/rehearsal.log; exit 1; }
tail -1 $out/rehearsal.log
for bt in "" "--backward-thread"; do
  tag=${bt:+_bt}
  h amoeba_n8_s56$tag --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6 $bt
  h amoeba_n2_s1$tag --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --stages 1 $bt
  h resnet_p4_s3$tag --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 3 $bt
  h resnet_p8_s7$tag --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 7 $bt
done
