#!/bin/bash
# r6s: PMC of the U-Net p1 step (bench headline): MFMA busy and waits (pass A), LDS traffic
# and bank conflicts (pass B) of the Winograd kernels
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r6s
mkdir -p $out
A="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $A --output-format csv -d $out/a -o run -- python3 bench.py --steps 1 --warmup 1 --sections none > $out/a.log 2>&1 || { echo "pass A failed"; tail -5 $out/a.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $B --output-format csv -d $out/b -o run -- python3 bench.py --steps 1 --warmup 1 --sections none > $out/b.log 2>&1 || { echo "pass B failed"; tail -5 $out/b.log; exit 1; }
for f in $out/a/run_counter_collection.csv $out/b/run_counter_collection.csv; do python3 scripts/r5/pmc_table.py $f; done > $out/pmc_table.txt
rm -f $out/a/run_kernel_trace.csv $out/b/run_kernel_trace.csv
cat $out/pmc_table.txt
