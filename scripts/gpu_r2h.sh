set -o pipefail
mkdir -p gpurun_out/r2h
timeout -k 10 200 python bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r2h/unet.log 2>&1 || exit 1
grep 'warmup step 1' gpurun_out/r2h/unet.log; tail -1 gpurun_out/r2h/unet.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/profile_bench.sh unet_r2 --gpus 1 --steps 4 --warmup 2 || exit 1
head -30 gpurun_out/prof_unet_r2/summary.md
