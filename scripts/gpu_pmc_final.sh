set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc5
for spec in "fwd4 40 256 256 48" "fwd4 40 64 64 192" "fwd4nf 40 1024 1024 12" "wgrad4 40 256 256 48" "wgrad4nf 40 1024 1024 12"; do
  set -- $spec; op=$1; shift; tag=${op}_$1_$2_$3_$4
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc5/$tag -o run -- python3 benchmarks/conv_probe.py --shape $1 $2 $3 $4 --op $op --iters 10 > gpurun_out/pmc5/$tag.log 2>&1 || exit 1
done
echo DONE
