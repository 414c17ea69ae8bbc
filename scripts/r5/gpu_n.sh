#!/bin/bash
# r5n: AmoebaNet stages are launch-bound now: does capping split-K (fewer reduction
# launches, TGPIPE_CG_SPLIT_CAP) pay?  n8m32 stage 6, n2m32 stage 1, eager as bench.py runs them
export TMPDIR=/tmp
out=gpurun_out/r5n
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; grep '"stage"' $out/$name.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('$name', d['stage'], 'dev', d['device_ms'], 'host', d['host_ms'])"; }
for cap in 0 4 2 1; do
  TGPIPE_CG_SPLIT_CAP=$cap h n8_s6_cap$cap --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 6
  TGPIPE_CG_SPLIT_CAP=$cap h n2_s1_cap$cap --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --stages 1
done
