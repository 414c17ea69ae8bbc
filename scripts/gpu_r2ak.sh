set -o pipefail
mkdir -p gpurun_out/r2ak
for v in 6 18 6 18; do
  timeout -k 10 300 env TGPIPE_F4_FUSED_VARIANT=$v python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2ak/unet_$v.log 2>&1 || exit 1
  echo "v$v $(tail -1 gpurun_out/r2ak/unet_$v.log | cut -c1-130)"
done
