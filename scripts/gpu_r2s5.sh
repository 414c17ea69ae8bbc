# Add the strided 3x3 implicit-GEMM shapes (AmoebaNet stem / reduction cells) to the plan
# table, then re-measure the AmoebaNet first step.
set -o pipefail
mkdir -p gpurun_out/s5
cp torchgpipe_amd/tuned/conv_gemm_mi355x.txt gpurun_out/s5/plans_before.txt
timeout -k 10 500 python benchmarks/tune_plans.py --merge --out gpurun_out/s5/conv_gemm_mi355x.txt > gpurun_out/s5/tune.log 2>&1 || { tail -20 gpurun_out/s5/tune.log; exit 1; }
tail -3 gpurun_out/s5/tune.log
cp gpurun_out/s5/conv_gemm_mi355x.txt torchgpipe_amd/tuned/conv_gemm_mi355x.txt
timeout -k 10 200 python benchmarks/first_step.py --model amoebanet --top 25 > gpurun_out/s5/first_amoeba.log 2>&1 || { tail -20 gpurun_out/s5/first_amoeba.log; exit 1; }
grep -E "^(build|step|plans)" gpurun_out/s5/first_amoeba.log
