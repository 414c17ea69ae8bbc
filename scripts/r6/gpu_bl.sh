#!/bin/bash
# r6bl: ResNet pipeline-1 lanes on the final tree: both (default), recompute only, none
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6bl
mkdir -p $out
run() { tag=$1; shift; timeout -k 10 400 python -u bench.py --model resnet --sections none "$@" > $out/b_$tag.json 2> $out/b_$tag.err || { tail -20 $out/b_$tag.err; exit 1; }; python3 -c "
import json;d=json.loads(open('$out/b_$tag.json').read().splitlines()[-1]);print('$tag', d['value'])"; }
for r in 1 2; do
  run both_$r || exit 1
  run rec_only_$r --overlap-forward off || exit 1
  run none_$r --overlap-forward off --overlap-recompute off || exit 1
done
