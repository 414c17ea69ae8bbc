# kernel-level durations (rocprofv3 kernel trace) of tgpipe implicit GEMM vs MIOpen, small grids
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2p
for spec in "fwd 1024 7 1024 1 1" "bwd 1024 7 1024 1 1" "wgrad 1024 7 1024 1 1" "fwd 256 7 256 1 7" "fwd 512 14 512 1 1" "wgrad 256 28 256 1 1"; do
  set -- $spec; tag=$1_$2_$3_$4_$5x$6
  for impl in ours miopen; do
    extra=""; [ $impl = miopen ] && extra="--miopen"
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r2p/${tag}_$impl -o run -- python3 benchmarks/convgemm_probe.py --x 20 $2 $3 $3 --co $4 --k $5 $6 --mode $1 --iters 20 $extra > gpurun_out/r2p/${tag}_$impl.log 2>&1 || exit 1
  done
done
find gpurun_out/r2p -name '*kernel_stats.csv' | sort | while read f; do echo "== $f"; head -6 "$f" | cut -c1-200; done
