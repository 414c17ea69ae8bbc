set -o pipefail
timeout -k 10 300 python benchmarks/stage_harness.py --model unet --balance 22 26 25 24 25 36 42 41 --chunks 40 --batch 640 --out gpurun_out/stage_p8_f4b.json > gpurun_out/stage_p8_f4b.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/stage_harness.py --model unet --balance 42 54 59 86 --chunks 16 --batch 512 --out gpurun_out/stage_p4_f4b.json > gpurun_out/stage_p4_f4b.log 2>&1 || exit 1
timeout -k 10 300 python benchmarks/stage_harness.py --model unet --balance 99 142 --chunks 32 --batch 512 --out gpurun_out/stage_p2_f4b.json > gpurun_out/stage_p2_f4b.log 2>&1 || exit 1
echo DONE
