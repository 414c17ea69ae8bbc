#!/bin/bash
# r5u: kernel traces of the slowest ResNet stages after the split-K models (p8 stage 7 at
# 36-image micro-batches, p4 stage 3 at 22)
export TMPDIR=/tmp
out=gpurun_out/r5u
mkdir -p $out
summ() {  # dir steps ms_per_step name
  python3 scripts/r4/rocpd_summary.py $1/run_results.db --last-ms $3 --steps $2 --top 30 > $out/$4.md && rm -rf $1
  head -14 $out/$4.md
}
hs() {  # name steps harness-args...
  name=$1; st=$2; shift 2
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/p_$name -o run -- python3 benchmarks/stage_harness.py --steps $st "$@" --out $out/h_$name.json > $out/$name.log 2>&1 || { tail -20 $out/$name.log; exit 1; }
  ms=$(python3 -c "import json;d=json.load(open('$out/h_$name.json'));print(d['stages'][0]['wall_ms']*$st)")
  summ $out/p_$name $st $ms $name
}
hs resnet_p8_s7 1 --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 7
hs resnet_p4_s3 1 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 3
