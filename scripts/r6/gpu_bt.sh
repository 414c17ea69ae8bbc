#!/bin/bash
# r6bt: ConvBN2d route memoised: whole GPU suite, then ResNet stage host / device time with
# and without (TGPIPE_ROUTE_CACHE), interleaved twice, and bench.py --model resnet
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6bt
mkdir -p $out
bash scripts/r6/gpu_r.sh || exit 1
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
for r in 1 2; do
  for v in 1 0; do
    TGPIPE_ROUTE_CACHE=$v h p4_${v}_$r --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 1 3 || exit 1
    TGPIPE_ROUTE_CACHE=$v h p8_${v}_$r --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 7 || exit 1
  done
done
for v in 1 0; do
  TGPIPE_ROUTE_CACHE=$v timeout -k 10 400 python -u bench.py --model resnet --sections none > $out/b_$v.json 2> $out/b_$v.err || { tail -20 $out/b_$v.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('$out/b_$v.json').read().splitlines()[-1]);print('route_cache=$v resnet p1', d['value'])"
done
