#!/bin/bash
# r5x: launch-bound AmoebaNet stages: multi-stream cells (3 / 2) vs one stream (0)
export TMPDIR=/tmp
out=gpurun_out/r5x
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
for cs in 0 2 3; do
  h n8_s56_cs$cs --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6 --cell-streams $cs
  h n2_s1_cs$cs --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --stages 1 --cell-streams $cs
done
timeout -k 10 300 python -u benchmarks/host_cell.py --out $out/host_cell_before.json > $out/host_cell.log 2>&1 || { tail -20 $out/host_cell.log; exit 1; }
cat $out/host_cell_before.json
h resnet_p4_s3 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 3
