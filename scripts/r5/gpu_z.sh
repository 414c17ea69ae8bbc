#!/bin/bash
# r5z: AmoebaNet cells with direct stream switches: numerics (GPU model tests + shared-GPU
# rehearsal), host cost, stage harness
export TMPDIR=/tmp
out=gpurun_out/r5z
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/models tests/distributed/test_shared_gpu_rehearsal.py tests/test_segments.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python -u benchmarks/host_cell.py --out $out/host_cell.json > $out/host_cell.log 2>&1 || { tail -20 $out/host_cell.log; exit 1; }
cat $out/host_cell.json
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
h n8_s56 --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6
h n2_s1 --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --stages 1
