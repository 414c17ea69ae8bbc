# Layer profile (micro-batch 16) + stage harness of the current bench balances: bash scripts/gpu_layerprof.sh <tag>
set -o pipefail
timeout -k 10 400 python benchmarks/layer_profile.py --model unet --micro-batch 16 --out gpurun_out/unet_layer_profile_$1.json > gpurun_out/layer_prof_$1.log 2>&1 || exit 1
bash scripts/gpu_stages.sh $1 "22 23 25 30 22 36 44 39" "45 55 59 82" "102 139" || exit 1
