#!/bin/bash
# r6ag: whole GPU suite + smoke on the tree with the merged BatchNorm allocations, then
# bench.py N=1 with the driver's defaults
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6ag
mkdir -p $out
bash scripts/r6/gpu_r.sh || exit 1
timeout -k 10 500 python -u bench.py > $out/bench_n1.json 2> $out/bench_n1.err || { tail -20 $out/bench_n1.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$out/bench_n1.json').read().splitlines()[-1])
print('unet', d['value'], 'base', d['baseline']['value'], 'gpipe', d['gpipe']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'], d['resnet101']['baseline']['value'])"
