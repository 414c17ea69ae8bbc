#!/bin/bash
# r6ac: CFG 12 (single-buffered 64 x 64 split-bf16 tile, two sub-stages per barrier): fp64
# tests, then the per-shape sweep against CFG 11 at ResNet's 22 / 36-image micro-batches and
# AmoebaNet's 40
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6ac
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ops/test_convbn_gpu.py tests/ops/test_group_convbn_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for mb in 22 36; do
  timeout -k 10 400 python -u benchmarks/convgemm_sweep.py --set resnet --micro-batch $mb --reps 10 --out $out/sweep_resnet_$mb.json > $out/sweep_resnet_$mb.log 2>&1 || { tail -20 $out/sweep_resnet_$mb.log; exit 1; }
done
timeout -k 10 600 python -u benchmarks/convgemm_sweep.py --set amoebanet --micro-batch 40 --reps 10 --out $out/sweep_amoeba_40.json > $out/sweep_amoeba_40.log 2>&1 || { tail -20 $out/sweep_amoeba_40.log; exit 1; }
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob('gpurun_out/r6ac/sweep_*.json')):
    rows = json.load(open(f))
    wins = sum(1 for r in rows if 'cfg12_us' in r and r['cfg12_us'] < min(r.get(f'cfg{c}_us', 1e9) for c in (7, 9, 10, 11)))
    ratio = [round(r['cfg11_us'] / r['cfg12_us'], 2) for r in rows if 'cfg12_us' in r and 'cfg11_us' in r]
    print(f, 'rows', len(rows), 'cfg12 best-of-emu', wins, 'cfg11/cfg12', ratio)
PY
