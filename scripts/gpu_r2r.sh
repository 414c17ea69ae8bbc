# PMC counters of the implicit-GEMM kernel at forced plans (one counter pass per run)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2r
run() {  # tag, pmc list, probe args...
  local tag=$1 pmc=$2; shift 2
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $pmc --output-format csv -d gpurun_out/r2r/$tag -o run -- python3 benchmarks/convgemm_probe.py "$@" --iters 10 > gpurun_out/r2r/$tag.log 2>&1
}
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for spec in "wg64 --x 20 64 28 28 --co 256 --mode wgrad --force 0 62" "fwd1024 --x 20 1024 7 7 --co 1024 --mode fwd --force 0 1" "fwd1024s3 --x 20 1024 7 7 --co 1024 --mode fwd --force 0 3"; do
  set -- $spec; tag=$1; shift
  run ${tag}_p1 "$P1" "$@" || exit 1
  run ${tag}_p2 "$P2" "$@" || exit 1
done
echo DONE
