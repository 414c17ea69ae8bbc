# Tap-gather cost of the 1x7 / 7x1 implicit-GEMM convolutions vs equal-GEMM 1x1 ones.
set -o pipefail
mkdir -p gpurun_out/s10
timeout -k 10 300 python benchmarks/gemm_equiv.py gpurun_out/s10/gemm_equiv.json > gpurun_out/s10/ge.log 2>&1 || { tail -20 gpurun_out/s10/ge.log; exit 1; }
cat gpurun_out/s10/ge.log
