#!/bin/bash
# r6bc: ResNet pipeline-1 and its baseline with and without the Winograd output-pass
# BatchNorm statistics (TGPIPE_BG_BN_STATS), interleaved twice on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6bc
mkdir -p $out
for r in 1 2; do
  for v in 1 0; do
    TGPIPE_BG_BN_STATS=$v timeout -k 10 400 python -u bench.py --sections resnet > $out/b_${v}_$r.json 2> $out/b_${v}_$r.err || { tail -20 $out/b_${v}_$r.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('$out/b_${v}_$r.json').read().splitlines()[-1])
print('stats=$v rep $r resnet', d['resnet101']['value'], d['resnet101']['baseline']['value'])"
  done
done
