# PMC counters of the implicit-GEMM conv kernel on representative AmoebaNet shapes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_cg
for spec in "fwd 1024 28 256 1 1" "fwd 1024 7 1024 1 1" "fwd 256 28 256 1 1" "wgrad 256 28 256 1 1" "fwd 64 28 64 1 7" "bwd 1024 28 256 1 1"; do
  set -- $spec; tag=$1_$2_$3_$4_$5x$6
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_cg/$tag -o run -- python3 benchmarks/convgemm_probe.py --x 20 $2 $3 $3 --co $4 --k $5 $6 --mode $1 --iters 10 > gpurun_out/pmc_cg/$tag.log 2>&1 || exit 1
done
echo DONE
