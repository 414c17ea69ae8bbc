#!/bin/bash
# r5o: per-shape AmoebaNet convolutions at micro-batch 40, tuned split-bf16 plans vs MIOpen
export TMPDIR=/tmp
out=gpurun_out/r5o
mkdir -p $out
timeout -k 10 900 python -u benchmarks/convbn_bench.py --micro-batch 40 --out $out/convbn_bench_n40.json > $out/convbn.log 2>&1 || { tail -20 $out/convbn.log; exit 1; }
tail -5 $out/convbn.log
