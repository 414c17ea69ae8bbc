set -o pipefail
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash scripts/rehearse_multirank.sh 2 8 || exit 1
timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 3 --warmup 2 > gpurun_out/amoeba_p1.log 2>&1 || exit 1
tail -1 gpurun_out/amoeba_p1.log | cut -c1-200
