# Stage harness runs for candidate balances: bash scripts/gpu_stages.sh <tag> "<p8 balance>" "<p4 balance>" "<p2 balance>"
set -o pipefail
tag=$1
timeout -k 10 300 python benchmarks/stage_harness.py --model unet --balance $2 --chunks 40 --batch 640 --out gpurun_out/stage_p8_$tag.json > gpurun_out/stage_p8_$tag.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/stage_harness.py --model unet --balance $3 --chunks 16 --batch 512 --out gpurun_out/stage_p4_$tag.json > gpurun_out/stage_p4_$tag.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/stage_harness.py --model unet --balance $4 --chunks 32 --batch 512 --out gpurun_out/stage_p2_$tag.json > gpurun_out/stage_p2_$tag.log 2>&1 || exit 1
echo DONE
