#!/bin/bash
# r6d: GPipe forward lanes, CFG 11 and the small-plane 3x3 implicit-GEMM route (tests),
# then the implicit-GEMM plan table re-tuned with CFG 10 / 11 among the candidates (and the
# 3x3 route's shapes), A/B against the shipped table on the AmoebaNet / ResNet stages and
# the N=1 bench, then the 3x3 route on the ResNet stages.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6d
mkdir -p $out
timeout -k 10 120 python -u scripts/debug/gpipe_lanes_diag.py > $out/lanes_diag.log 2>&1; cat $out/lanes_diag.log | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/models/test_resnet_fused_gpu.py \
    tests/ops/test_convbn_gpu.py -k "not cfg or cfg11" > $out/tests.log 2>&1 \
  && tail -1 $out/tests.log || { tail -30 $out/tests.log; exit 1; }
TGPIPE_GEMM3X3_MAX_PLANE=196 timeout -k 10 1100 python -u benchmarks/tune_plans.py \
    --out $out/conv_gemm_mi355x.txt --lib-out $out/lib_dgrad_mi355x.txt > $out/tune.log 2>&1 \
  || { tail -20 $out/tune.log; exit 1; }
tail -2 $out/tune.log
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
for db in shipped new; do
  if [ $db = new ]; then export TGPIPE_CG_DB=$out/conv_gemm_mi355x.txt TGPIPE_LIB_DGRAD_DB=$out/lib_dgrad_mi355x.txt; fi
  h n8_s56_$db --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6 || exit 1
  h n2_s1_$db --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --stages 1 || exit 1
  h resnet_p8_s7_$db --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 7 || exit 1
  h resnet_p4_s23_$db --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 2 3 || exit 1
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 10 --warmup 3 > $out/bench_$db.json 2> $out/bench_$db.err || { tail -20 $out/bench_$db.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$out/bench_$db.json').read().splitlines()[-1]);print('bench $db unet', d['value'], 'gpipe', d['gpipe']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'], d['resnet101']['baseline']['value'])"
done
export TGPIPE_GEMM3X3_MAX_PLANE=196
h resnet_p8_s7_g3 --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 7 || exit 1
h resnet_p4_s23_g3 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 2 3 || exit 1
