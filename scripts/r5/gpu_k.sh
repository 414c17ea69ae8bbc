#!/bin/bash
# r5k: re-tune the plan tables with ResNet micro-batches 22 / 36 (reference pipeline-4 / -8)
# and the split-bf16 heuristic, then ResNet p4 stage 2 / p8 stage 7 with the new tables
export TMPDIR=/tmp
out=gpurun_out/r5k
mkdir -p $out
timeout -k 10 1000 python -u benchmarks/tune_plans.py --out $out/conv_gemm_mi355x.txt \
    --lib-out $out/lib_dgrad_mi355x.txt > $out/tune.log 2>&1 || { echo "tune failed"; tail -20 $out/tune.log; exit 1; }
tail -3 $out/tune.log
export TGPIPE_CG_DB=$out/conv_gemm_mi355x.txt TGPIPE_LIB_DGRAD_DB=$out/lib_dgrad_mi355x.txt
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; grep '"stage"' $out/$name.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$name', d['stage'], 'dev', d['device_ms'], 'host', d['host_ms'])"; }
h resnet_p4 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632
h resnet_p8 --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400
