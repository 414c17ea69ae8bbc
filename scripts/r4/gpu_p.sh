# Memory-side PMC of the implicit-GEMM kernels on AmoebaNet 7x7 / 14x14 shapes at micro-batch
# 40: L2 hit rate, L1->L2 read requests, HBM fetch bytes.
set -o pipefail
out=gpurun_out/r4p
mkdir -p $out
export TMPDIR=/tmp
for spec in "fwd 1024 7 1024 1 1" "fwd 4096 7 1024 1 1" "fwd 512 14 512 1 1" "bwd 1024 7 1024 1 1"; do
  set -- $spec; tag=$1_$2_$3_$4_$5x$6
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_l2/$tag -o run -- python3 benchmarks/convgemm_probe.py --x 40 $2 $3 $3 --co $4 --k $5 $6 --mode $1 --iters 10 > $out/l2_$tag.log 2>&1 || { tail $out/l2_$tag.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_fetch/$tag -o run -- python3 benchmarks/convgemm_probe.py --x 40 $2 $3 $3 --co $4 --k $5 $6 --mode $1 --iters 10 > $out/fetch_$tag.log 2>&1 || { tail $out/fetch_$tag.log; exit 1; }
done
echo DONE
