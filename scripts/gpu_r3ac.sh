# Round 3: U-Net p1 kernel trace of the current tree (headline config).
set -o pipefail
bash scripts/profile_bench.sh unet_p1_r3 --gpus 1 --steps 4 --warmup 2 --sections none || exit 1
head -40 gpurun_out/prof_unet_p1_r3/summary.md
