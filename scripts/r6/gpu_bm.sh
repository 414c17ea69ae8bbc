#!/bin/bash
# r6bm: step-cache scan cached per cache epoch: whole GPU suite, then ResNet / U-Net bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6bm
mkdir -p $out
bash scripts/r6/gpu_r.sh || exit 1
for r in 1 2; do
  timeout -k 10 500 python -u bench.py > $out/bench_n1_$r.json 2> $out/bench_n1_$r.err || { tail -20 $out/bench_n1_$r.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('$out/bench_n1_$r.json').read().splitlines()[-1])
print('unet', d['value'], 'base', d['baseline']['value'], 'gpipe', d['gpipe']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'], d['resnet101']['baseline']['value'])"
done
