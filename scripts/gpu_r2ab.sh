set -o pipefail
mkdir -p gpurun_out/r2ab
timeout -k 10 300 python -u benchmarks/amoeba_op_profile.py --chunks 4 --batch 80 --rows 40 > gpurun_out/r2ab/ops.log 2>&1 || { tail -20 gpurun_out/r2ab/ops.log; exit 1; }
head -60 gpurun_out/r2ab/ops.log | cut -c1-220
