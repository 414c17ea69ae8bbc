#!/bin/bash
# r6bg: where ResNet pipeline-1's GPU idles (bench.py --model resnet, 2 steps traced)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${R6BG_OUT:-r6bg}
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/p_resnet -o run -- python3 bench.py --gpus 1 --model resnet --steps 2 --warmup 3 --sections none > $out/resnet_p1.json 2> $out/resnet_p1.err || { tail -20 $out/resnet_p1.err; exit 1; }
ms=$(python3 -c "import json;d=json.loads(open('$out/resnet_p1.json').read().splitlines()[-1]);print(d['ms_per_step']*2)")
python3 scripts/r6/gaps.py $out/p_resnet/run_results.db --last-ms $ms --top 30 > $out/gaps.txt && rm -rf $out/p_resnet
cat $out/gaps.txt
