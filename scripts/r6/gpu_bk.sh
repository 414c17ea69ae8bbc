#!/bin/bash
# r6bk: ResNet p4 / p8 every stage eager and with captured cells, and the no-GPipe baseline,
# on one box (final tree) -- the ResNet prediction rows
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6bk
mkdir -p $out
timeout -k 10 400 python -u bench.py --sections resnet > $out/bench_resnet.json 2> $out/bench_resnet.err || { tail -20 $out/bench_resnet.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$out/bench_resnet.json').read().splitlines()[-1])
print('resnet p1', d['resnet101']['value'], 'baseline', d['resnet101']['baseline']['value'])"
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([s['device_ms'] for s in d['stages']])")"; }
h resnet_p4 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 || exit 1
h resnet_p4_gc --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --graph-cells || exit 1
h resnet_p8 --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 || exit 1
h resnet_p8_gc --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --graph-cells || exit 1
