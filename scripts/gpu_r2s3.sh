# First-step host profile (AmoebaNet) and U-Net stage harness at the reference p2/p4/p8 balances.
set -o pipefail
mkdir -p gpurun_out/s3
timeout -k 10 200 python benchmarks/first_step.py --model amoebanet > gpurun_out/s3/first_amoeba.log 2>&1 || { tail -20 gpurun_out/s3/first_amoeba.log; exit 1; }
head -4 gpurun_out/s3/first_amoeba.log
timeout -k 10 300 python benchmarks/stage_harness.py --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 --out gpurun_out/s3/harness_p8_ref.json > gpurun_out/s3/h8.log 2>&1 || { tail -20 gpurun_out/s3/h8.log; exit 1; }
cat gpurun_out/s3/h8.log
timeout -k 10 300 python benchmarks/stage_harness.py --balance 30 66 84 61 --chunks 16 --batch 512 --out gpurun_out/s3/harness_p4_ref.json > gpurun_out/s3/h4.log 2>&1 || { tail -20 gpurun_out/s3/h4.log; exit 1; }
cat gpurun_out/s3/h4.log
timeout -k 10 300 python benchmarks/stage_harness.py --balance 104 137 --chunks 32 --batch 512 --out gpurun_out/s3/harness_p2_ref.json > gpurun_out/s3/h2.log 2>&1 || { tail -20 gpurun_out/s3/h2.log; exit 1; }
cat gpurun_out/s3/h2.log
