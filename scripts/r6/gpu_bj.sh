#!/bin/bash
# r6bj: ResNet pipeline-1 with captured cells vs the default (lanes), interleaved twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6bj
mkdir -p $out
for r in 1 2; do
  for v in on auto; do
    timeout -k 10 400 python -u bench.py --model resnet --graph-cells $v --sections none > $out/b_${v}_$r.json 2> $out/b_${v}_$r.err || { tail -20 $out/b_${v}_$r.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('$out/b_${v}_$r.json').read().splitlines()[-1])
print('graph_cells=$v rep $r', d['value'], d['ms_per_step'], d.get('config'))" | cut -c1-200
  done
done
