#!/bin/bash
# r5a: split-bf16 implicit-GEMM configurations 7-9: fp64 numerics, then the plan sweep at
# micro-batch 40 (AmoebaNet n*m32 shapes).
export TMPDIR=/tmp
out=gpurun_out/r5a
mkdir -p $out
timeout -k 10 500 python -u -m pytest -q --timeout 240 --timeout-method thread \
    tests/ops/test_convbn_gpu.py -k "cfg7 or cfg8 or cfg9" > $out/test.log 2>&1
rc=$?
tail -5 $out/test.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u benchmarks/convgemm_sweep.py --micro-batch 40 --reps 20 \
    --out $out/sweep40.json > $out/sweep.log 2>&1
echo "sweep rc=$?"
