# Plan tuner on the final round-4 GEMM loop (8-wave tile interleaving included).
set -o pipefail
out=gpurun_out/r4z
mkdir -p $out
timeout -k 10 900 python -u benchmarks/tune_plans.py --out $out/conv_gemm_mi355x.txt --lib-out $out/lib_dgrad_mi355x.txt > $out/tune.log 2>&1 || { tail -20 $out/tune.log; exit 1; }
tail -3 $out/tune.log
