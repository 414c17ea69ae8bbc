#!/bin/bash
# r5ag: last-stage direct backward: GPU tests of the engine paths, then the last stages
export TMPDIR=/tmp
out=gpurun_out/r5ag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_segments.py tests/distributed tests/test_step_graph.py tests/test_gpu_pipeline.py tests/test_checkpoint.py tests/models -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms'], s['peak_mem_gib']) for s in d['stages']])")"; }
h n2_s1 --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --stages 1
h n8_s7 --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 7
h resnet_p4_s3 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 3
h unet_p4_s3 --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 3
