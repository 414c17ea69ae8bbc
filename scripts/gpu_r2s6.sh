# Host enqueue vs device time per step: AmoebaNet n1m32 and U-Net p1 (stage harness).
set -o pipefail
mkdir -p gpurun_out/s6
timeout -k 10 300 python benchmarks/stage_harness.py --model amoebanet --balance 24 --chunks 32 --batch 640 --out gpurun_out/s6/harness_amoeba_n1.json > gpurun_out/s6/ha.log 2>&1 || { tail -20 gpurun_out/s6/ha.log; exit 1; }
grep stage gpurun_out/s6/ha.log
timeout -k 10 300 python benchmarks/stage_harness.py --model amoebanet --balance 9 15 --chunks 32 --batch 1280 --out gpurun_out/s6/harness_amoeba_n2.json > gpurun_out/s6/ha2.log 2>&1 || { tail -20 gpurun_out/s6/ha2.log; exit 1; }
grep stage gpurun_out/s6/ha2.log
timeout -k 10 300 python benchmarks/stage_harness.py --balance 241 --chunks 2 --batch 80 --out gpurun_out/s6/harness_unet_p1.json > gpurun_out/s6/hu.log 2>&1 || { tail -20 gpurun_out/s6/hu.log; exit 1; }
grep stage gpurun_out/s6/hu.log
