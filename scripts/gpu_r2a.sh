# Round-2 first GPU call: AmoebaNet kernel profile, first-step cost, RCCL same-GPU probe.
set -o pipefail
mkdir -p gpurun_out/r2a
bash scripts/profile_bench.sh amoeba_n1m32 --model amoebanet --gpus 1 --steps 3 --warmup 2 || exit 1
tail -1 gpurun_out/prof_amoeba_n1m32/bench.log | cut -c1-300
for k in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 3 --warmup 2 > gpurun_out/r2a/unet_run$k.log 2>&1 || exit 1
  grep 'warmup step 1' gpurun_out/r2a/unet_run$k.log
done
du -sh ~/.cache/miopen 2>/dev/null; ls ~/.cache/miopen/* 2>/dev/null | head
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/rccl_same_gpu_probe.py > gpurun_out/r2a/rccl_probe.log 2>&1
echo "rccl probe rc=$?"; tail -20 gpurun_out/r2a/rccl_probe.log
