#!/bin/bash
# r6bd: ResNet p4 / p8 stage harness three times on the final tree (per-stage median)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6bd
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([s['device_ms'] for s in d['stages']])")"; }
for r in 1 2 3; do
  h resnet_p4_$r --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 || exit 1
  h resnet_p8_$r --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 || exit 1
done
