#!/bin/bash
# r6i: ResNet p8 stage 7 / p4 stage 3 with and without the BatchNorm gradient-accumulation
# fusion, interleaved (host-bound stages: box-to-box host speed differs)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6i
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
for rep in 1 2; do
  for acc in 1 0; do
    TGPIPE_BN_GRAD_ACCUM=$acc h p8s7_acc${acc}_$rep --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 7 || exit 1
    TGPIPE_BN_GRAD_ACCUM=$acc h p4s3_acc${acc}_$rep --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 3 || exit 1
  done
done
