#!/bin/bash
# r5ar: the fused split-K BatchNorm on 12^2 - 14^2 planes too (TGPIPE_SPLIT_BN=2): numerics,
# then stage harness / n1m32 bench A/B against 7^2-only (TGPIPE_SPLIT_BN=1)
export TMPDIR=/tmp
out=gpurun_out/r5ar
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/ops/test_convbn_gpu.py tests/ops/test_group_convbn_gpu.py tests/models -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
for sb in 1 2; do
  export TGPIPE_SPLIT_BN=$sb
  h n8_s56_sb$sb --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6
  h n8_s3_sb$sb --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 3
  h n2_s1_sb$sb --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --stages 1
  timeout -k 10 400 python3 bench.py --gpus 1 --model amoebanet --steps 5 --warmup 3 --sections none > $out/amoeba_n1_sb$sb.json 2> $out/amoeba_n1_sb$sb.err || { tail -20 $out/amoeba_n1_sb$sb.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/amoeba_n1_sb$sb.json'));print('n1m32 sb$sb', d['value'], d['ms_per_step'])"
done
