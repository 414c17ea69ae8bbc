#!/bin/bash
# r5e: with the split-bf16 batched GEMM, does moving the 64/128-channel U-Net layers off the
# fused F(4x4) kernel pay?  U-Net p1 at BG_MIN_CHANNELS 256 (shipped) / 128 / 64
export TMPDIR=/tmp
out=gpurun_out/r5e
mkdir -p $out
for mc in 256 128 64; do
  TGPIPE_WINOGRAD_BG_MIN_CHANNELS=$mc timeout -k 10 300 python -u bench.py --steps 5 --warmup 3 --sections none > $out/unet_p1_mc$mc.json 2> $out/unet_p1_mc$mc.log || { echo "bench mc=$mc failed"; tail -20 $out/unet_p1_mc$mc.log; exit 1; }
  python -c "import json;d=json.load(open('$out/unet_p1_mc$mc.json'));print($mc, d['value'], d['config']['rank0_peak_mem_gib'])"
done
