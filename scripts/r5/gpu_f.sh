#!/bin/bash
# r5f: can two RCCL ranks share the box's one GPU?
export TMPDIR=/tmp
out=gpurun_out/r5f
mkdir -p $out
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 scripts/rccl_same_gpu_probe.py > $out/probe.log 2>&1
echo "rc=$?"
tail -30 $out/probe.log
