#!/bin/bash
# r5ap: kernel traces of the latest tree (pre-split weights, fused small-plane split
# BatchNorm): AmoebaNet n1m32 (bench headline, captured cells) and n8m32 stage 6 (eager)
export TMPDIR=/tmp
out=gpurun_out/r5ap
mkdir -p $out
summ() {  # dir steps ms_per_step name
  python3 scripts/r4/rocpd_summary.py $1/run_results.db --last-ms $3 --steps $2 --top 30 > $out/$4.md && rm -rf $1
  head -14 $out/$4.md
}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/p_amoeba -o run -- python3 bench.py --gpus 1 --model amoebanet --steps 2 --warmup 3 --sections none > $out/amoeba_n1.json 2> $out/amoeba_n1.err || { tail -20 $out/amoeba_n1.err; exit 1; }
ms=$(python3 -c "import json;d=json.load(open('$out/amoeba_n1.json'));print(d['ms_per_step']*2)")
summ $out/p_amoeba 2 $ms amoeba_n1m32
hs() {  # name steps harness-args...
  name=$1; st=$2; shift 2
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/p_$name -o run -- python3 benchmarks/stage_harness.py --steps $st "$@" --out $out/h_$name.json > $out/$name.log 2>&1 || { tail -20 $out/$name.log; exit 1; }
  ms=$(python3 -c "import json;d=json.load(open('$out/h_$name.json'));print(d['stages'][0]['wall_ms']*$st)")
  summ $out/p_$name $st $ms $name
}
hs amoeba_n8m32_s6 2 --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 6
