# Host cost of an AmoebaNet n1 step: micro-batches of 1-2 images make the kernels tiny, so
# the host enqueue time is the launch overhead itself.
set -o pipefail
mkdir -p gpurun_out/s7
timeout -k 10 300 python benchmarks/stage_harness.py --model amoebanet --balance 24 --chunks 32 --batch 32 --out gpurun_out/s7/harness_amoeba_mb1.json > gpurun_out/s7/h1.log 2>&1 || { tail -20 gpurun_out/s7/h1.log; exit 1; }
grep stage gpurun_out/s7/h1.log
timeout -k 10 300 python benchmarks/stage_harness.py --model amoebanet --balance 24 --chunks 32 --batch 160 --out gpurun_out/s7/harness_amoeba_mb5.json > gpurun_out/s7/h5.log 2>&1 || { tail -20 gpurun_out/s7/h5.log; exit 1; }
grep stage gpurun_out/s7/h5.log
