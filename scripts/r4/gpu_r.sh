# Plan tuner with the round-4 GEMM tiles (CFG 6 included), then a larger 8-GPU U-Net
# (48,608) for the maximum-size search.
set -o pipefail
out=gpurun_out/r4r
mkdir -p $out
timeout -k 10 900 python -u benchmarks/tune_plans.py --out $out/conv_gemm_mi355x.txt --lib-out $out/lib_dgrad_mi355x.txt > $out/tune.log 2>&1 || { tail -20 $out/tune.log; exit 1; }
tail -3 $out/tune.log
timeout -k 10 600 python -u benchmarks/memory.py unet -B 48 -C 608 --balance 852 123 32 32 35 33 35 991 --chunks 128 --out $out/memory_unet_48_608_p8.json > $out/memory_608.log 2>&1 || { tail -20 $out/memory_608.log; exit 1; }
tail -1 $out/memory_608.log
