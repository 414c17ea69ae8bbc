# rocprofv3 PMC passes over the Winograd forward kernel (benchmarks/conv_probe.py).
# Usage: OP=fwd4 bash scripts/pmc_wino.sh <outdir> "N C K H" ...   (OP: fwd, wgrad, fwd4, wgrad4)
set -o pipefail
out=$1; shift
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for shape in "$@"; do
  tag=${OP:-fwd}_$(echo $shape | tr ' ' _)
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $out/p1_$tag -o run -- python3 benchmarks/conv_probe.py --shape $shape --op ${OP:-fwd} --iters 10 > $out/p1_$tag.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD TCC_HIT_sum TCC_MISS_sum --output-format csv -d $out/p2_$tag -o run -- python3 benchmarks/conv_probe.py --shape $shape --op ${OP:-fwd} --iters 10 > $out/p2_$tag.log 2>&1 || exit 1
done
