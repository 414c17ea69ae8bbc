#!/bin/bash
# r5ax: PMC of the split-bf16 implicit GEMM with and without the pre-split weights
# (TGPIPE_CG_PRESPLIT_MB=0: in-kernel split) on the r5b shapes (AmoebaNet mb 40)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r5ax
mkdir -p $out
A="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"
for mb in 0 2048; do
  for spec in "fwd 512 14 512 9 1" "fwd 1024 7 1024 7 1" "bwd 512 14 512 9 1"; do
    set -- $spec; tag=ps${mb}_$1_$2_$3_$4_cfg$5
    TGPIPE_CG_PRESPLIT_MB=$mb timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $A --output-format csv -d $out/$tag -o run -- python3 benchmarks/convgemm_probe.py --x 40 $2 $3 $3 --co $4 --mode $1 --iters 10 --force $5 $6 > $out/$tag.log 2>&1 || { echo "fail $tag"; tail -5 $out/$tag.log; exit 1; }
  done
done
for f in $out/*/run_counter_collection.csv; do echo "== $f"; python3 scripts/r5/pmc_table.py $f; done > $out/pmc_table.txt
cat $out/pmc_table.txt
