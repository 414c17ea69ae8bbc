# conv GEMM planner sweep: blocks-per-launch targets
set -o pipefail
mkdir -p gpurun_out/r2d
for cfg in "200 200 400 512" "400 200 400 512" "200 1000 1000 512" "400 1000 1000 1024" "100000 1000 1000 512"; do
  set -- $cfg
  tag="fb$1_fs$2_ts$3_tw$4"
  TGPIPE_CG_FILL_BIG=$1 TGPIPE_CG_FILL_SMALL=$2 TGPIPE_CG_TARGET_SMALL=$3 TGPIPE_CG_TARGET_WGRAD=$4 \
    timeout -k 10 300 python benchmarks/convbn_bench.py --micro-batch 20 --out gpurun_out/r2d/cb_$tag.json > gpurun_out/r2d/cb_$tag.log 2>&1 || exit 1
  echo "$tag $(tail -1 gpurun_out/r2d/cb_$tag.log)"
done
