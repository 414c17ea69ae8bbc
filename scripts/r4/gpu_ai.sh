# Every kernel of one fused ReLU-Conv-BN op (forward + backward, one stream) on AmoebaNet
# shapes at micro-batch 40: what the BatchNorm / reduction passes cost beside the GEMMs.
set -o pipefail
out=gpurun_out/r4ai
mkdir -p $out
export TMPDIR=/tmp
for spec in "1024 7 1024 1 1" "512 14 512 1 1" "256 28 256 1 1" "256 7 256 1 7"; do
  set -- $spec; tag=$1_$2_$3_$4x$5
  timeout -k 10 120 rocprofv3 --kernel-trace -d $out/p_$tag -o run -- python3 benchmarks/convbn_probe.py --x 40 $1 $2 $2 --co $3 --k $4 $5 --iters 12 > $out/$tag.log 2>&1 || { tail -20 $out/$tag.log; exit 1; }
  python3 scripts/r4/rocpd_summary.py $out/p_$tag/run_results.db --last-ms 100000 --steps 12 --top 14 > $out/summary_$tag.md && rm -rf $out/p_$tag
  echo "== $tag"; head -16 $out/summary_$tag.md
done
