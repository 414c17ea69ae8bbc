#!/bin/bash
# r6bh: cProfile of ResNet p4 stage 3 (host-paced) on the final tree
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6bh
mkdir -p $out
timeout -k 10 600 python -u -m cProfile -o $out/resnet_p4_s3.prof benchmarks/stage_harness.py --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 3 --warmup 2 --steps 1 > $out/resnet.log 2>&1 || { tail -20 $out/resnet.log; exit 1; }
python3 -c "
import pstats
p = pstats.Stats('$out/resnet_p4_s3.prof')
p.sort_stats('tottime').print_stats(35)
" > $out/tottime.txt
python3 -c "
import pstats
p = pstats.Stats('$out/resnet_p4_s3.prof')
p.sort_stats('cumulative').print_stats(45)
" > $out/cumtime.txt
rm -f $out/resnet_p4_s3.prof
head -70 $out/tottime.txt | tail -45
