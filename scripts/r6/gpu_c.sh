#!/bin/bash
# r6c: CFG 10 (single-buffered 8-wave split-bf16 tile, two workgroups per CU): fp64 tests,
# per-shape A/B against CFG 9 (AmoebaNet at micro-batch 40, ResNet at 22), then AmoebaNet
# n1m32 with every CFG 9 plan run as CFG 10 against the shipped plans.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6c
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/ops/test_convbn_gpu.py -k "cfg10 or (presplit and 10)" > $out/tests.log 2>&1 \
  && tail -1 $out/tests.log \
  && timeout -k 10 300 python -u benchmarks/convgemm_sweep.py --micro-batch 40 --reps 20 \
       --out $out/sweep_amoeba40.json > $out/sweep_amoeba40.log 2>&1 \
  && timeout -k 10 300 python -u benchmarks/convgemm_sweep.py --set resnet --micro-batch 22 \
       --reps 20 --out $out/sweep_resnet22.json > $out/sweep_resnet22.log 2>&1 \
  && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --overlap-recompute off \
       --overlap-forward off --sections gpipe > $out/bench_nolanes.json 2> $out/bench_nolanes.log \
  && timeout -k 10 300 python -u bench.py --model amoebanet --steps 10 --warmup 3 \
       > $out/amoeba_cfg9.json 2> $out/amoeba_cfg9.log \
  && TGPIPE_CG_SINGLE=1 timeout -k 10 300 python -u bench.py --model amoebanet --steps 10 \
       --warmup 3 > $out/amoeba_cfg10.json 2> $out/amoeba_cfg10.log \
  && python - <<'PY'
import json
for f in ('sweep_amoeba40', 'sweep_resnet22'):
    for r in json.load(open(f'gpurun_out/r6c/{f}.json')):
        print(r['shape'], r['mode'], 'best', r['best_us'], r['top'][0][:2], 'cfg9',
              r.get('cfg9_us'), 'cfg10', r.get('cfg10_us'))
for f in ('amoeba_cfg9', 'amoeba_cfg10'):
    print(f, json.loads(open(f'gpurun_out/r6c/{f}.json').read().splitlines()[-1])['value'])
PY
rc=$?
tail -3 $out/tests.log
exit $rc
