#!/bin/bash
# r6ai: per-kernel times of the BatchNorm kernels, new (two loads in flight) vs previous
# build: kernel traces of one AmoebaNet n1m32 step and one ResNet p4 stage-3 step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6ai
mkdir -p $out
cp torchgpipe_amd/_C.so /tmp/_C_new.so
for v in new old; do
  if [ $v = new ]; then cp /tmp/_C_new.so torchgpipe_amd/_C.so; else cp torchgpipe_amd/_C_old.so torchgpipe_amd/_C.so; fi
  for m in n1 p4; do
    if [ $m = n1 ]; then args="--model amoebanet --balance 24 --chunks 32 --batch 1280"; else args="--model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 3"; fi
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/p_$m$v -o run -- python3 benchmarks/stage_harness.py --steps 1 $args --out $out/h_$m$v.json > $out/$m$v.log 2>&1 || { tail -20 $out/$m$v.log; exit 1; }
    ms=$(python3 -c "import json;d=json.load(open('$out/h_$m$v.json'));print(d['stages'][0]['wall_ms'])")
    python3 scripts/r4/rocpd_summary.py $out/p_$m$v/run_results.db --last-ms $ms --steps 1 --top 60 > $out/${m}_$v.md && rm -rf $out/p_$m$v
    head -1 $out/${m}_$v.md
    grep -E "bn_|split_bn" $out/${m}_$v.md
  done
done
