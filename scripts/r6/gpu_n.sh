#!/bin/bash
# r6n: would forward lanes pay on ResNet-101's small-micro-batch stages?  (running
# statistics off so the stage is lane-eligible; scripts/r6/resnet_lanes_probe.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6n
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u scripts/r6/resnet_lanes_probe.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
for l in auto on; do
  h p4s3_$l --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 2 3 --lanes $l || exit 1
  h p8s7_$l --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 6 7 --lanes $l || exit 1
done
