#!/bin/bash
# r5c: re-tune the implicit-GEMM plan tables with the split-bf16 configurations, then
# AmoebaNet n1m32 (bench.py --model amoebanet) with the new tables vs the shipped ones.
export TMPDIR=/tmp
out=gpurun_out/r5c
mkdir -p $out
timeout -k 10 900 python -u benchmarks/tune_plans.py --out $out/conv_gemm_mi355x.txt \
    --lib-out $out/lib_dgrad_mi355x.txt > $out/tune.log 2>&1 || { echo "tune failed"; tail -20 $out/tune.log; exit 1; }
tail -3 $out/tune.log
TGPIPE_CG_DB=$out/conv_gemm_mi355x.txt TGPIPE_LIB_DGRAD_DB=$out/lib_dgrad_mi355x.txt \
  timeout -k 10 400 python -u bench.py --model amoebanet --steps 5 --warmup 3 > $out/amoeba_new.json 2> $out/amoeba_new.log || { echo "bench new failed"; tail -20 $out/amoeba_new.log; exit 1; }
cat $out/amoeba_new.json
timeout -k 10 400 python -u bench.py --model amoebanet --steps 5 --warmup 3 > $out/amoeba_old.json 2> $out/amoeba_old.log || { echo "bench old failed"; exit 1; }
cat $out/amoeba_old.json
