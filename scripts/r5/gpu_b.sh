#!/bin/bash
# r5b: PMC of the split-bf16 implicit GEMM vs the f32 one on two AmoebaNet mb-40 shapes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r5b
mkdir -p $out
A="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"
B="SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
for spec in "fwd 512 14 512 9 1" "fwd 512 14 512 4 1" "fwd 1024 7 1024 7 1" "fwd 1024 7 1024 6 1"; do
  set -- $spec; tag=$1_$2_$3_$4_cfg$5
  for pass in A B; do
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc ${!pass} --output-format csv -d $out/$tag$pass -o run -- python3 benchmarks/convgemm_probe.py --x 40 $2 $3 $3 --co $4 --mode $1 --iters 10 --force $5 $6 > $out/$tag$pass.log 2>&1 || { echo "fail $tag $pass"; tail -5 $out/$tag$pass.log; exit 1; }
  done
done
echo DONE
