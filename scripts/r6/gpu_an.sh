#!/bin/bash
# r6an: strided Conv-BN choice timed per geometry at the pipeline micro-batch
# (TGPIPE_STRIDED_CHOICE=1) vs the shipped set measured at pipeline-1's 110 images:
# kernel traces of ResNet p4 stages 2 and 3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6an
mkdir -p $out
for st in 3 2; do
  for v in shipped timed; do
    if [ $v = timed ]; then export TGPIPE_STRIDED_CHOICE=1; else unset TGPIPE_STRIDED_CHOICE; fi
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/p_$st$v -o run -- python3 benchmarks/stage_harness.py --steps 1 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages $st --out $out/h_$st$v.json > $out/$st$v.log 2>&1 || { tail -20 $out/$st$v.log; exit 1; }
    ms=$(python3 -c "import json;d=json.load(open('$out/h_$st$v.json'));print(d['stages'][0]['wall_ms'])")
    python3 scripts/r4/rocpd_summary.py $out/p_$st$v/run_results.db --last-ms $ms --steps 1 --top 60 > $out/p4_s${st}_$v.md && rm -rf $out/p_$st$v
    echo "stage $st $v: $(head -1 $out/p4_s${st}_$v.md)"
  done
done
