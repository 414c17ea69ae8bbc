#!/bin/bash
# r6h: AmoebaNet captured-cell stage harness (n8m32 crashed at its second stage with the
# capture streams shared across stages), then the kernel traces (gpu_g.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6f
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([s['device_ms'] for s in d['stages']])")"; }
h amoeba_n8m32_gc --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --graph-cells || exit 1
h amoeba_n4m32_gc --model amoebanet --balance 3 6 7 8 --chunks 32 --batch 1152 --graph-cells || exit 1
bash scripts/r6/gpu_pmc.sh || exit 1
bash scripts/r6/gpu_g.sh
