set -o pipefail
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 3 --warmup 2 > gpurun_out/amoeba_p1.log 2>&1 || { tail -5 gpurun_out/amoeba_p1.log; exit 1; }
tail -1 gpurun_out/amoeba_p1.log | cut -c1-260
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 3 --warmup 2 --channels-last > gpurun_out/amoeba_p1_cl.log 2>&1 || { tail -5 gpurun_out/amoeba_p1_cl.log; exit 1; }
tail -1 gpurun_out/amoeba_p1_cl.log | cut -c1-260
