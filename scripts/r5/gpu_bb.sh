#!/bin/bash
# r5bb: U-Net p4 stage 1 (the p4 bottleneck, device-bound) under the engine's options: lanes
# off, captured cells; AmoebaNet n4m32 with captured cells
export TMPDIR=/tmp
out=gpurun_out/r5bb
mkdir -p $out
h() { name=$1; shift; timeout -k 10 900 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms'], s.get('graph_phase')) for s in d['stages']])")"; }
h unet_p4_s1 --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 1
h unet_p4_s1_nolanes --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 1 --lanes off
h unet_p4_s1_gc --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 1 --graph-cells --warmup 4
h amoeba_n4m32_gc --model amoebanet --balance 3 6 7 8 --chunks 32 --batch 1152 --graph-cells --warmup 4 --steps 2
