# Kernel traces (with device-idle accounting) of the AmoebaNet n1m32 and U-Net p1 benches.
set -o pipefail
bash scripts/profile_bench.sh amoeba_s2 --model amoebanet --gpus 1 --steps 3 --warmup 2 || exit 1
bash scripts/profile_bench.sh unet_s2 --gpus 1 --steps 4 --warmup 2 || exit 1
head -24 gpurun_out/prof_amoeba_s2/summary.md; head -6 gpurun_out/prof_unet_s2/summary.md
