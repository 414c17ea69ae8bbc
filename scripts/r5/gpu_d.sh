#!/bin/bash
# r5d: split-bf16 batched-GEMM Winograd numerics, bg_bench A/B, U-Net p1 bench
export TMPDIR=/tmp
out=gpurun_out/r5d
mkdir -p $out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread \
    tests/ops/test_winograd_gpu.py -k "batched_gemm or split_bf16" > $out/test.log 2>&1
rc=$?
tail -15 $out/test.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for emu in 0 1; do
  TGPIPE_BG_EMU=$emu timeout -k 10 300 python -u bench.py --steps 5 --warmup 3 --sections none > $out/unet_p1_emu$emu.json 2> $out/unet_p1_emu$emu.log || { echo "bench emu=$emu failed"; tail -20 $out/unet_p1_emu$emu.log; exit 1; }
  cat $out/unet_p1_emu$emu.json
done
