#!/bin/bash
# r6bf: kernel traces of the final round-6 tree: AmoebaNet n1m32 (bench, captured cells), U-Net p1
# (bench headline), ResNet p4 stage 3 and AmoebaNet n8m32 stage 6 (stage harness, eager)
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r6bf
mkdir -p $out
summ() {  # dir steps ms_per_step name
  python3 scripts/r4/rocpd_summary.py $1/run_results.db --last-ms $3 --steps $2 --top 30 > $out/$4.md && rm -rf $1
  head -14 $out/$4.md
}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/p_amoeba -o run -- python3 bench.py --gpus 1 --model amoebanet --steps 2 --warmup 3 --sections none > $out/amoeba_n1.json 2> $out/amoeba_n1.err || { tail -20 $out/amoeba_n1.err; exit 1; }
ms=$(python3 -c "import json;d=json.loads(open('$out/amoeba_n1.json').read().splitlines()[-1]);print(d['ms_per_step']*2)")
summ $out/p_amoeba 2 $ms amoeba_n1m32
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/p_unet -o run -- python3 bench.py --gpus 1 --steps 3 --warmup 3 --sections none > $out/unet_p1.json 2> $out/unet_p1.err || { tail -20 $out/unet_p1.err; exit 1; }
ms=$(python3 -c "import json;d=json.loads(open('$out/unet_p1.json').read().splitlines()[-1]);print(d['ms_per_step']*3)")
summ $out/p_unet 3 $ms unet_p1
hs() {  # name steps harness-args...
  name=$1; st=$2; shift 2
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/p_$name -o run -- python3 benchmarks/stage_harness.py --steps $st "$@" --out $out/h_$name.json > $out/$name.log 2>&1 || { tail -20 $out/$name.log; exit 1; }
  ms=$(python3 -c "import json;d=json.load(open('$out/h_$name.json'));print(d['stages'][0]['wall_ms']*$st)")
  summ $out/p_$name $st $ms $name
}
hs resnet_p4_s3 1 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 3
hs amoeba_n8m32_s6 2 --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 6
# per-shape implicit GEMM (shipped plans) vs MIOpen over AmoebaNet-D(18,256) at micro-batch 40
timeout -k 10 600 python3 benchmarks/convbn_bench.py --micro-batch 40 --out $out/convbn_bench_n40.json > $out/convbn_bench.log 2>&1 || { tail -20 $out/convbn_bench.log; exit 1; }
tail -3 $out/convbn_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/p_resnet -o run -- python3 bench.py --gpus 1 --model resnet --steps 2 --warmup 3 --sections none > $out/resnet_p1.json 2> $out/resnet_p1.err || { tail -20 $out/resnet_p1.err; exit 1; }
ms=$(python3 -c "import json;d=json.loads(open('$out/resnet_p1.json').read().splitlines()[-1]);print(d['ms_per_step']*2)")
summ $out/p_resnet 2 $ms resnet_p1
