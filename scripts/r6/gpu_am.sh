#!/bin/bash
# r6am: F(4x4) weight-gradient variant rule (256-511 channels at <= 2048 tiles: non-fused;
# 512 -> 256 at >= 4096 tiles: split-bf16): Winograd / ResNet / U-Net tests, a kernel trace
# of ResNet p4 stage 3 and U-Net p1 stage times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6am
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ops/test_winograd_gpu.py tests/ops/test_unet_ops_gpu.py tests/models/test_resnet_fused_gpu.py tests/test_gpu_pipeline.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/p -o run -- python3 benchmarks/stage_harness.py --steps 1 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 3 --out $out/h.json > $out/p4.log 2>&1 || { tail -20 $out/p4.log; exit 1; }
ms=$(python3 -c "import json;d=json.load(open('$out/h.json'));print(d['stages'][0]['wall_ms'])")
python3 scripts/r4/rocpd_summary.py $out/p/run_results.db --last-ms $ms --steps 1 --top 40 > $out/p4_s3.md && rm -rf $out/p
head -1 $out/p4_s3.md
grep -E "wgrad" $out/p4_s3.md
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
h u1 --model unet --balance 241 --chunks 2 --batch 80 || exit 1
h u4 --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 1 2 || exit 1
