#!/bin/bash
# r6v: bench.py at N=8 as a shared-GPU rehearsal (gloo, host-staged messages: functional
# only, not a measurement) -- every section, the ResNet / AmoebaNet lanes and slots included
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6v
mkdir -p $out
timeout -k 20 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --steps 2 --warmup 1 --section-steps 1 --backend gloo > $out/bench_n8.json 2> $out/bench_n8.err; rc=$?
tail -3 $out/bench_n8.err
python3 -c "
import json
d=json.loads(open('$out/bench_n8.json').read().splitlines()[-1])
print('lines', len(open('$out/bench_n8.json').read().splitlines()), 'sections', d.get('section_s'))
for k in ('baseline','amoebanet','resnet101','tuned','striped','amoebanet_graph_cells'):
    v=d.get(k); print(k, None if v is None else {kk: v[kk] for kk in ('value','error') if kk in v})
"
exit $rc
