#!/bin/bash
# r6q: ResNet stages and bench N=1 with the slot views cached (runstats.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6q
mkdir -p $out
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
h p4s23 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 2 3 || exit 1
h p8s67 --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 6 7 || exit 1
h p4s23_reclanes --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 2 3 --lanes off || exit 1
timeout -k 10 500 python -u bench.py --sections resnet > $out/bench_resnet.json 2> $out/bench_resnet.err || { tail -20 $out/bench_resnet.err; exit 1; }
python -c "
import json;d=json.loads(open('$out/bench_resnet.json').read().splitlines()[-1])
print('resnet', d['resnet101']['value'], d['resnet101']['baseline']['value'])"
