#!/bin/bash
# Functional rehearsal of the multi-rank bench on ONE GPU: N ranks share cuda:0,
# messages go through host memory over gloo (bench.py --backend gloo).
# Not a measurement; checks that every stage of the real U-Net/AmoebaNet
# partitions runs and the JSON line comes out.
set -e -o pipefail
mkdir -p gpurun_out/rehearsal
port=29611
for n in "$@"; do
  for model in unet amoebanet; do
    port=$((port + 1))
    if [ "$model" = unet ]; then extra="--batch $((16 * n)) --chunks $((2 * n))"; else extra="--batch $((8 * n)) --chunks $((2 * n))"; fi
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
      --master-addr 127.0.0.1 --master-port "$port" bench.py --gpus "$n" --steps 2 --warmup 1 \
      --backend gloo --model "$model" $extra \
      > "gpurun_out/rehearsal/${model}_n${n}.json" 2> "gpurun_out/rehearsal/${model}_n${n}.err"
    echo "n=$n $model ok: $(cut -c1-160 gpurun_out/rehearsal/${model}_n${n}.json)"
  done
done
