#!/bin/bash
# r5ad: split-bf16 batched-GEMM F(4x4) weight gradient (variant 2): numerics, then timing
# against the fused / non-fused f32 kernels on the U-Net / ResNet shapes
export TMPDIR=/tmp
out=gpurun_out/r5ad
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/ops/test_winograd_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 400 python -u benchmarks/wgrad_variants.py --out $out/wgrad_variants.json \
  --shape 40 512 512 24 --shape 40 1024 1024 12 --shape 16 512 512 24 --shape 16 1024 1024 12 \
  --shape 16 2048 2048 6 --shape 40 256 256 48 --shape 16 256 256 48 --shape 40 128 128 96 \
  --shape 22 256 256 14 --shape 36 512 512 7 --shape 110 256 256 14 --shape 40 2048 2048 6 \
  --all-f4 > $out/wgrad.log 2>&1 || { tail -20 $out/wgrad.log; exit 1; }
cat $out/wgrad.log
