# ResNet strided Conv-BN geometries on the fused native op: fp64 tests, ResNet-101 p1 x2.
set -o pipefail
out=gpurun_out/r4ae
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/models/test_resnet_fused_gpu.py -q -x --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --model resnet --gpus 1 --steps 20 --warmup 4 --sections none > $out/resnet_$rep.json 2> $out/resnet_$rep.err || { tail -20 $out/resnet_$rep.err; exit 1; }
  TGPIPE_STRIDED_CHOICE=0 python -c "import json;d=json.load(open('$out/resnet_$rep.json'));print('resnet p1', d['value'])"
done
