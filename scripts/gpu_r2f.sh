set -o pipefail
mkdir -p gpurun_out/r2f
timeout -k 10 600 python -u -m pytest tests/ops/test_convbn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2f/test_convbn.log 2>&1
rc=$?; tail -5 gpurun_out/r2f/test_convbn.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1073741824 256 200 200 400 512" "512 256 200 200 400 512" "1073741824 256 200 1000 1000 512" "512 512 200 600 800 1024" "1073741824 256 200 200 400 1024"; do
  set -- $cfg
  tag="mk$1_tb$2_fb$3_fs$4_ts$5_tw$6"
  TGPIPE_CG_BIGSPLIT_MINK=$1 TGPIPE_CG_TARGET_BIG=$2 TGPIPE_CG_FILL_BIG=$3 TGPIPE_CG_FILL_SMALL=$4 TGPIPE_CG_TARGET_SMALL=$5 TGPIPE_CG_TARGET_WGRAD=$6 \
    timeout -k 10 300 python benchmarks/convbn_bench.py --micro-batch 20 --out gpurun_out/r2f/cb_$tag.json > gpurun_out/r2f/cb_$tag.log 2>&1 || exit 1
  echo "$tag $(tail -1 gpurun_out/r2f/cb_$tag.log)"
done
