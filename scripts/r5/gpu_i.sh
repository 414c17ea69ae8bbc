#!/bin/bash
# r5i: captured cells vs eager on the host-bound stages (ResNet p4 stage 2, p8 stage 7,
# AmoebaNet n8m32 stages 5 / 6)
export TMPDIR=/tmp
out=gpurun_out/r5i
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; grep '"stage"' $out/$name.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$name', d['stage'], 'dev', d['device_ms'], 'host', d['host_ms'], 'launch', d['graph_launch_ms'], 'mem', d['peak_mem_gib'])"; }
h resnet_p4_gc --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 2 --graph-cells
h resnet_p8_gc --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 7 --graph-cells
h amoeba_n8m32_gc --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6 --graph-cells
