#!/bin/bash
# r6y: ResNet-101 p4 / p8 stage harness, every stage, with the lanes (bench default now)
# and without any lanes (round 5's ResNet default was recompute lanes only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6y
mkdir -p $out
h() { name=$1; shift; timeout -k 10 900 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
h resnet_p4 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 || exit 1
h resnet_p8 --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 || exit 1
h resnet_p4_reconly --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --lanes off || exit 1
h resnet_p8_reconly --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --lanes off || exit 1
