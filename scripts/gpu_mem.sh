# Memory benchmark in the shipped configuration (Winograd caches on, budgeted; fused ops)
set -o pipefail
mkdir -p gpurun_out/mem
run() { tag=$1; shift; timeout -k 10 560 python -u benchmarks/memory.py "$@" --out gpurun_out/mem/$tag.json > gpurun_out/mem/$tag.log 2>&1 || { tail -5 gpurun_out/mem/$tag.log; exit 1; }; tail -1 gpurun_out/mem/$tag.log | cut -c1-300; }
case $1 in
  a) run unet_48_160_p8 unet --experiment pipeline-8
     run amoebanet_72_512_p8 amoebanet --experiment pipeline-8 ;;
  b) run unet_24_300_p1 unet -B 24 -C 300 --balance 1077 --chunks 32 ;;
  c) run unet_48_576_p8 unet -B 48 -C 576 --balance 852 123 32 32 35 33 35 991 --chunks 128 ;;
esac
