#!/bin/bash
# r6ab: AmoebaNet-D(18,256) n1m32 (bench amoebanet section) under its engine options, one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6ab
mkdir -p $out
run() { tag=$1; shift; timeout -k 10 400 env "$@" python -u bench.py --model amoebanet --sections none --steps 5 --warmup 2 > $out/$tag.json 2> $out/$tag.err || { tail -20 $out/$tag.err; exit 1; }; echo "$tag $(python3 -c "import json;d=json.loads(open('$out/$tag.json').read().splitlines()[-1]);print(d['value'])")"; }
run default TGPIPE_X=0 || exit 1
run streams2 TGPIPE_CELL_STREAMS=2 || exit 1
run streams4 TGPIPE_CELL_STREAMS=4 || exit 1
run default_b TGPIPE_X=0 || exit 1
