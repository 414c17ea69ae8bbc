#!/bin/bash
# r6bo: bench.py N=1 with the warmed-up objects frozen out of Python's cyclic GC vs not
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6bo
mkdir -p $out
for r in 1 2; do
  for v in 1 0; do
    TGPIPE_GC_FREEZE=$v timeout -k 10 500 python -u bench.py > $out/b_${v}_$r.json 2> $out/b_${v}_$r.err || { tail -20 $out/b_${v}_$r.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('$out/b_${v}_$r.json').read().splitlines()[-1])
print('freeze=$v rep $r unet', d['value'], 'base', d['baseline']['value'], 'gpipe', d['gpipe']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'], d['resnet101']['baseline']['value'])"
  done
done
