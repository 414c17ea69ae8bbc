# Device-only (hipGraph-timed) implicit-GEMM convolution times vs MIOpen and hipBLASLt.
set -o pipefail
mkdir -p gpurun_out/s11
timeout -k 10 400 python benchmarks/gemm_device_time.py gpurun_out/s11/gemm_device.json > gpurun_out/s11/gd.log 2>&1 || { tail -20 gpurun_out/s11/gd.log; exit 1; }
cat gpurun_out/s11/gd.log
