#!/bin/bash
# r6bq: bench.py N=1 with 2 vs 3 warm-up steps (the third step still grows the caching
# allocator's pools: benchmarks/diag/alloc_probe.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6bq
mkdir -p $out
for r in 1 2; do
  for w in 3 2; do
    timeout -k 10 500 python -u bench.py --warmup $w > $out/b_w${w}_$r.json 2> $out/b_w${w}_$r.err || { tail -20 $out/b_w${w}_$r.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('$out/b_w${w}_$r.json').read().splitlines()[-1])
print('warmup=$w rep $r unet', d['value'], 'base', d['baseline']['value'], 'gpipe', d['gpipe']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'], d['resnet101']['baseline']['value'])"
  done
done
