#!/bin/bash
# r6ap: strided Conv-BN choice timed at the pipeline micro-batch (TGPIPE_STRIDED_CHOICE=1)
# vs the shipped set: kernel traces of the other ResNet stages holding a stride-2 block
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6ap
mkdir -p $out
run() { tag=$1; shift; for v in shipped timed; do
    if [ $v = timed ]; then export TGPIPE_STRIDED_CHOICE=1; else unset TGPIPE_STRIDED_CHOICE; fi
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/p_$tag$v -o run -- python3 benchmarks/stage_harness.py --steps 1 "$@" --out $out/h_$tag$v.json > $out/$tag$v.log 2>&1 || { tail -20 $out/$tag$v.log; return 1; }
    ms=$(python3 -c "import json;d=json.load(open('$out/h_$tag$v.json'));print(d['stages'][0]['wall_ms'])")
    python3 scripts/r4/rocpd_summary.py $out/p_$tag$v/run_results.db --last-ms $ms --steps 1 --top 60 > $out/${tag}_$v.md && rm -rf $out/p_$tag$v
    echo "$tag $v: $(head -1 $out/${tag}_$v.md)"
  done; }
run p4s1 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 1 || exit 1
run p8s7 --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 7 || exit 1
run p8s2 --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 2 || exit 1
run p8s3 --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 3 || exit 1
