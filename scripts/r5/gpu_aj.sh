#!/bin/bash
# r5aj: per-shape A/B of the pre-split weights (AmoebaNet-D(18,256) convolutions at
# micro-batch 40: forward / backward-data / weight-gradient device time)
export TMPDIR=/tmp
out=gpurun_out/r5aj
mkdir -p $out
for mb in 0 512; do
  TGPIPE_CG_PRESPLIT_MB=$mb timeout -k 10 400 python -u benchmarks/convbn_bench.py --micro-batch 40 --out $out/convbn_bench_n40_ps$mb.json > $out/ps$mb.log 2>&1 || { tail -20 $out/ps$mb.log; exit 1; }
  tail -1 $out/ps$mb.log
done
