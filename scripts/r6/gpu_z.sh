#!/bin/bash
# r6z: final-tree bench.py N=1 (driver defaults) twice, then a kernel trace of ResNet p4
# stage 3 without lanes (the configuration bench.py runs at N=4)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6z
mkdir -p $out
for r in 1 2; do
  timeout -k 10 500 python -u bench.py > $out/bench_n1_$r.json 2> $out/bench_n1_$r.err || { tail -20 $out/bench_n1_$r.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('$out/bench_n1_$r.json').read().splitlines()[-1])
print('unet', d['value'], 'base', d['baseline']['value'], 'gpipe', d['gpipe']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'], d['resnet101']['baseline']['value'])"
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/p_res -o run -- python3 benchmarks/stage_harness.py --steps 1 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 3 --out $out/h_res.json > $out/res.log 2>&1 || { tail -20 $out/res.log; exit 1; }
ms=$(python3 -c "import json;d=json.load(open('$out/h_res.json'));print(d['stages'][0]['wall_ms'])")
python3 scripts/r4/rocpd_summary.py $out/p_res/run_results.db --last-ms $ms --steps 1 --top 30 > $out/resnet_p4_s3_nolanes.md && rm -rf $out/p_res
head -3 $out/resnet_p4_s3_nolanes.md
