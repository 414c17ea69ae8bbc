#!/bin/bash
# r6aj: the split-bf16 Winograd input image with 2 / 1 channels per thread on small grids:
# Winograd / ResNet / U-Net op tests, then kernel traces (ResNet p4 stage 3) and stage
# times, new vs previous build (shipped as torchgpipe_amd/_C_old.so) on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r6aj
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ops/test_winograd_gpu.py tests/ops/test_unet_ops_gpu.py tests/models/test_resnet_fused_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
cp torchgpipe_amd/_C.so /tmp/_C_new.so
for v in new old; do
  if [ $v = new ]; then cp /tmp/_C_new.so torchgpipe_amd/_C.so; else cp torchgpipe_amd/_C_old.so torchgpipe_amd/_C.so; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/p_$v -o run -- python3 benchmarks/stage_harness.py --steps 1 --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 3 --out $out/h_$v.json > $out/p4$v.log 2>&1 || { tail -20 $out/p4$v.log; exit 1; }
  ms=$(python3 -c "import json;d=json.load(open('$out/h_$v.json'));print(d['stages'][0]['wall_ms'])")
  python3 scripts/r4/rocpd_summary.py $out/p_$v/run_results.db --last-ms $ms --steps 1 --top 40 > $out/p4_$v.md && rm -rf $out/p_$v
  head -1 $out/p4_$v.md
  grep -E "bg_" $out/p4_$v.md
done
h() { name=$1; shift; timeout -k 10 600 python -u benchmarks/stage_harness.py "$@" --out $out/stage_harness_$name.json > $out/$name.log 2>&1 || { echo "harness $name failed"; tail -20 $out/$name.log; exit 1; }; echo "$name $(python -c "import json;d=json.load(open('$out/stage_harness_$name.json'));print([(s['device_ms'], s['host_ms']) for s in d['stages']])")"; }
for rep in 1 2; do
  for v in new old; do
    if [ $v = new ]; then cp /tmp/_C_new.so torchgpipe_amd/_C.so; else cp torchgpipe_amd/_C_old.so torchgpipe_amd/_C.so; fi
    h p4_${v}_$rep --model resnet101 --balance 44 92 124 110 --chunks 256 --batch 5632 --stages 2 3 || exit 1
    h p8_${v}_$rep --model resnet101 --balance 26 22 33 44 44 66 66 69 --chunks 150 --batch 5400 --stages 6 7 || exit 1
    h u1_${v}_$rep --model unet --balance 241 --chunks 2 --batch 80 || exit 1
  done
done
cp /tmp/_C_new.so torchgpipe_amd/_C.so
