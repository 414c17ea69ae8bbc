#!/bin/bash
# r6ba: BatchNorm statistics from the batched-GEMM Winograd output pass: Winograd / ResNet
# tests, kernel traces of ResNet p4 stages 1 / 3, bench.py N=1
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6ba
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ops/test_winograd_gpu.py tests/models/test_resnet_fused_gpu.py tests/test_overlap_recompute.py tests/test_gpu_pipeline.py > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for st in 2 3; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/p_$st -o run -- python3 benchmarks/stage_harness.py --steps 1 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages $st --out $out/h_$st.json > $out/s$st.log 2>&1 || { tail -20 $out/s$st.log; exit 1; }
  ms=$(python3 -c "import json;d=json.load(open('$out/h_$st.json'));print(d['stages'][0]['wall_ms'])")
  python3 scripts/r4/rocpd_summary.py $out/p_$st/run_results.db --last-ms $ms --steps 1 --top 60 > $out/p4_s${st}.md && rm -rf $out/p_$st
  echo "stage $st: $(head -1 $out/p4_s${st}.md)"
  grep -E "bn_stats|bg_output" $out/p4_s${st}.md
done
timeout -k 10 500 python -u bench.py > $out/bench_n1.json 2> $out/bench_n1.err || { tail -20 $out/bench_n1.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$out/bench_n1.json').read().splitlines()[-1])
print('unet', d['value'], 'base', d['baseline']['value'], 'gpipe', d['gpipe']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'], d['resnet101']['baseline']['value'])"
