# Round 3: PMC passes over the batched-GEMM Winograd kernels (U-Net p4 stage-1/2 shapes) and
# the fused F(4x4) forward at 128 ch 96^2: MFMA busy, waits, LDS conflicts, L2 hit rate.
set -o pipefail
out=gpurun_out/r3ah
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD TCC_HIT_sum TCC_MISS_sum"
run() {  # tag, program args...
  tag=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $out/p1_$tag -o run -- python3 "$@" > $out/p1_$tag.log 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d $out/p2_$tag -o run -- python3 "$@" > $out/p2_$tag.log 2>&1 || return 1
}
run bg512 benchmarks/bg_probe.py --shape 32 512 512 24 --iters 10 || exit 1
run bg1024 benchmarks/bg_probe.py --shape 32 1024 1024 12 --iters 10 || exit 1
run bg256 benchmarks/bg_probe.py --shape 32 256 256 48 --iters 10 || exit 1
run f4_128 benchmarks/conv_probe.py --shape 32 128 128 96 --op fwd4 --iters 10 || exit 1
for t in bg512 bg1024 bg256; do
  python3 scripts/pmc_table.py $(find $out/p1_$t $out/p2_$t -name '*counter_collection.csv') --kernel bg_gemm > $out/pmc_$t.txt || exit 1
  cat $out/pmc_$t.txt
done
python3 scripts/pmc_table.py $(find $out/p1_f4_128 $out/p2_f4_128 -name '*counter_collection.csv') --kernel f4_conv > $out/pmc_f4_128.txt && cat $out/pmc_f4_128.txt
find $out -name '*.csv' -size +20M -delete
