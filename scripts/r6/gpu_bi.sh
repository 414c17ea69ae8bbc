#!/bin/bash
# r6bi: ResNet stages with captured cells vs eager on the final tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6bi
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
h p4_eager --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 2 3 || exit 1
h p4_gc --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 2 3 --graph-cells || exit 1
h p8_eager --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 6 7 || exit 1
h p8_gc --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 6 7 --graph-cells || exit 1
