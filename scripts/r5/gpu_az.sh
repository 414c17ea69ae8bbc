#!/bin/bash
# r5az: ResNet-101 p2 at the reference's B=25000 (m=1667 micro-batches of 15 images): stage 1
# is host-bound eagerly; how far do captured cells (PipelineStage(graph_cells=True), opt-in
# at N > 1) take both stages?  Plus ResNet p4 stage 2 / p8 stage 7 with captured cells.
export TMPDIR=/tmp
out=gpurun_out/r5az
mkdir -p $out
h() { name=$1; shift; timeout -k 10 900 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms'], s.get('graph_phase')) for s in d['stages']])")"; }
h resnet_p2_b25000_gc --model resnet101 --balance 135 235 --chunks 1667 --batch 25000 --checkpoint always --graph-cells --warmup 4 --steps 1
h resnet_p4_s2_gc --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 2 --graph-cells --warmup 4 --steps 2
