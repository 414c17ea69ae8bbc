# Memory benchmark on the round-4 tree (U-Net(48,160) p8, the largest 8-GPU U-Net (48,576) and
# 1-GPU U-Net (24,300), stage by stage), then the plan tuner for the interleaved GEMM loop.
set -o pipefail
out=gpurun_out/r4l
mkdir -p $out
m() {  # name, args...
  local name=$1; shift
  timeout -k 10 500 python -u benchmarks/memory.py unet "$@" --out $out/$name.json > $out/$name.log 2>&1 || { echo "$name failed"; tail -20 $out/$name.log; return 1; }
  echo "== $name"; tail -1 $out/$name.log
}
m memory_unet_48_160_p8 --experiment pipeline-8 || exit 1
m memory_unet_24_300_p1 -B 24 -C 300 --balance 1077 --chunks 32 || exit 1
m memory_unet_48_576_p8 -B 48 -C 576 --balance 852 123 32 32 35 33 35 991 --chunks 128 || exit 1
timeout -k 10 900 python -u benchmarks/tune_plans.py --out $out/conv_gemm_mi355x.txt --lib-out $out/lib_dgrad_mi355x.txt > $out/tune.log 2>&1 || { tail -20 $out/tune.log; exit 1; }
tail -3 $out/tune.log
