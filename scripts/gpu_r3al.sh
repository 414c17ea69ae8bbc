# Round 3: U-Net(5,64) per-layer stage times (every layer its own stage) at micro-batch 16
# (p2 / p8 experiments) and 32 (p4), 8 / 4 micro-batches per pass (times scale with the
# micro-batch count), for MI355X balances with the current kernels.
set -o pipefail
out=gpurun_out/r3al
mkdir -p $out
ones=$(python3 -c "print(' '.join(['1'] * 241))")
timeout -k 10 500 python benchmarks/stage_harness.py --balance $ones --chunks 8 --batch 128 --out $out/unet_layers_mb16.json > $out/mb16.log 2>&1 || { tail -20 $out/mb16.log; exit 1; }
grep -c stage $out/mb16.log
timeout -k 10 500 python benchmarks/stage_harness.py --balance $ones --chunks 4 --batch 128 --out $out/unet_layers_mb32.json > $out/mb32.log 2>&1 || { tail -20 $out/mb32.log; exit 1; }
grep -c stage $out/mb32.log
