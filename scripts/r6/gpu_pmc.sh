#!/bin/bash
# r6pmc: PMC of the 8-wave split-bf16 tile double-buffered (CFG 9) and single-buffered at
# two workgroups per CU (CFG 10) on the verdict's shapes (AmoebaNet micro-batch 40)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r6pmc
mkdir -p $out
A="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"
for cfg in 9 10; do
  for spec in "fwd 512 14 512 1" "fwd 1024 7 1024 1" "bwd 512 14 512 1" "bwd 1024 28 256 1"; do
    set -- $spec; tag=$1_$2_$3_$4_cfg$cfg
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $A --output-format csv -d $out/$tag -o run -- python3 benchmarks/convgemm_probe.py --x 40 $2 $3 $3 --co $4 --mode $1 --iters 10 --force $cfg $5 > $out/$tag.log 2>&1 || { echo "fail $tag"; tail -5 $out/$tag.log; exit 1; }
  done
done
for f in $out/*/run_counter_collection.csv; do echo "== $f"; python3 scripts/r5/pmc_table.py $f; done > $out/pmc_table.txt
cat $out/pmc_table.txt
