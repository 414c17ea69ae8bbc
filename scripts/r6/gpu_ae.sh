#!/bin/bash
# r6ae: AmoebaNet stages with micro-batch lanes (BatchNorm statistics slotted) instead of
# three-stream cells: the host-bound stages trade per-node stream switches for lanes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6ae
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
for rep in 1 2; do
  h n8_cells_$rep --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6 || exit 1
  h n8_lanes_$rep --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6 --cell-streams 0 --lanes on || exit 1
  h n2_cells_$rep --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --stages 1 || exit 1
  h n2_lanes_$rep --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --stages 1 --cell-streams 0 --lanes on || exit 1
done
