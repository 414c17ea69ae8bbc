set -o pipefail
mkdir -p gpurun_out/r2e
for cfg in "1073741824 256 200" "512 256 200" "512 512 200" "1024 256 200" "512 256 400"; do
  set -- $cfg
  tag="mk$1_tb$2_fb$3"
  TGPIPE_CG_BIGSPLIT_MINK=$1 TGPIPE_CG_TARGET_BIG=$2 TGPIPE_CG_FILL_BIG=$3 \
    timeout -k 10 300 python benchmarks/convbn_bench.py --micro-batch 20 --out gpurun_out/r2e/cb_$tag.json > gpurun_out/r2e/cb_$tag.log 2>&1 || exit 1
  echo "$tag $(tail -1 gpurun_out/r2e/cb_$tag.log)"
done
