#!/bin/bash
# r6br: HIP API calls of ResNet pipeline-1 steps (host-side blocking calls)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r6br
mkdir -p $out
timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace -d $out/p -o run -- python3 bench.py --gpus 1 --model resnet --steps 2 --warmup 3 --sections none > $out/resnet_p1.json 2> $out/resnet_p1.err || { tail -20 $out/resnet_p1.err; exit 1; }
ms=$(python3 -c "import json;d=json.loads(open('$out/resnet_p1.json').read().splitlines()[-1]);print(d['ms_per_step']*2)")
python3 scripts/r6/hip_api_long.py $out/p/run_results.db --last-ms $ms --top 25 > $out/api.txt; rc=$?
python3 scripts/r6/gaps.py $out/p/run_results.db --last-ms $ms --top 10 > $out/gaps.txt
rm -rf $out/p
cat $out/api.txt; head -8 $out/gaps.txt
exit $rc
