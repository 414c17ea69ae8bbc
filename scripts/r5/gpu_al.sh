#!/bin/bash
# r5al: U-Net p4 stage harness A/B of the Winograd path choice: batched-GEMM (split-bf16)
# from 128 / 64 channels instead of 256, and the fused F(4x4) slab-ring variant 18
export TMPDIR=/tmp
out=gpurun_out/r5al
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([s['device_ms'] for s in d['stages']])")"; }
h unet_p4 --model unet --balance 30 66 84 61 --chunks 16 --batch 512
TGPIPE_WINOGRAD_BG_MIN_CHANNELS=128 h unet_p4_bg128 --model unet --balance 30 66 84 61 --chunks 16 --batch 512
TGPIPE_WINOGRAD_BG_MIN_CHANNELS=64 h unet_p4_bg64 --model unet --balance 30 66 84 61 --chunks 16 --batch 512
TGPIPE_F4_FUSED_VARIANT=18 h unet_p4_v18 --model unet --balance 30 66 84 61 --chunks 16 --batch 512
