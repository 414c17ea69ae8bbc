#!/bin/bash
# r6l: the single-GPU memory maximum U-Net(24,300) on this round's tree, then bench.py N=1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6e gpurun_out/r6l
timeout -k 10 560 python -u benchmarks/memory.py unet -B 24 -C 300 --balance 1077 --chunks 32 --out gpurun_out/r6e/unet_24_300_p1.json > gpurun_out/r6e/unet_24_300_p1.log 2>&1 || { tail -5 gpurun_out/r6e/unet_24_300_p1.log; exit 1; }
tail -1 gpurun_out/r6e/unet_24_300_p1.log | cut -c1-300
timeout -k 10 500 python -u bench.py > gpurun_out/r6l/bench_n1.json 2> gpurun_out/r6l/bench_n1.err || { tail -20 gpurun_out/r6l/bench_n1.err; exit 1; }
tail -1 gpurun_out/r6l/bench_n1.json | cut -c1-600
