#!/bin/bash
# r6b: full GPU suite, then GPipe vs PipelineStage with the lanes off (same single stream),
# then the memory maxima (U-Net(24,300) p1, AmoebaNet-D(72,512) p8 with the breakdown).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6b
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > $out/gpu_tests.log 2>&1 \
  && tail -1 $out/gpu_tests.log \
  && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --overlap-recompute off \
       --overlap-forward off --sections gpipe > $out/bench_nolanes.json 2> $out/bench_nolanes.log \
  && tail -1 $out/bench_nolanes.json | cut -c1-200 \
  && timeout -k 10 560 python -u benchmarks/memory.py amoebanet --experiment pipeline-8 \
       --out $out/amoebanet_72_512_p8.json > $out/mem_amoeba.log 2>&1 \
  && tail -1 $out/mem_amoeba.log | cut -c1-400 \
  && timeout -k 10 560 python -u benchmarks/memory.py unet -B 24 -C 300 --balance 1077 --chunks 32 \
       --out $out/unet_24_300_p1.json > $out/mem_unet_p1.log 2>&1 \
  && tail -1 $out/mem_unet_p1.log | cut -c1-400
rc=$?
tail -3 $out/gpu_tests.log
exit $rc
