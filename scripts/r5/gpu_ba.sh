#!/bin/bash
# r5ba: AmoebaNet n2m32 / n8m32 stages with captured cells (opt-in at N > 1) on the final
# tree, for the prediction table's captured-cells rows
export TMPDIR=/tmp
out=gpurun_out/r5ba
mkdir -p $out
h() { name=$1; shift; timeout -k 10 900 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms'], s.get('graph_phase')) for s in d['stages']])")"; }
h amoeba_n2m32_gc --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --graph-cells --warmup 4 --steps 2
h amoeba_n8m32_gc --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --graph-cells --warmup 4 --steps 2
h amoeba_n2m1 --model amoebanet --balance 7 17 --chunks 1 --batch 96 --checkpoint always
