# multi-process rehearsal on one GPU (gloo transport, ranks share the device)
set -o pipefail
mkdir -p gpurun_out/r2aa
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --model amoebanet --steps 2 --warmup 1 --also-tuned no > gpurun_out/r2aa/amoeba_p2.log 2>&1 || { tail -20 gpurun_out/r2aa/amoeba_p2.log; exit 1; }
tail -1 gpurun_out/r2aa/amoeba_p2.log | cut -c1-300
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --backend gloo --steps 2 --warmup 1 --also-tuned no > gpurun_out/r2aa/unet_p4.log 2>&1 || { tail -20 gpurun_out/r2aa/unet_p4.log; exit 1; }
tail -1 gpurun_out/r2aa/unet_p4.log | cut -c1-300
