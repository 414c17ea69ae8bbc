# variant 20 check + bench, three-stream whole-step capture at m=1, AmoebaNet harness with
# graph-launch timing, default bench.
set -o pipefail
out=gpurun_out/r4f
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ops/test_winograd_gpu.py -k "split_patch" > $out/v20_tests.log 2>&1; rc=$?; tail -3 $out/v20_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u benchmarks/wino_variants.py --variants 6 20 --shape 32 128 128 96 --shape 40 128 128 96 --shape 16 128 128 96 --shape 40 64 64 192 --shape 16 64 64 192 --shape 32 64 64 192 --shape 16 128 64 192 --out $out/wino_v20.json > $out/wino_v20.log 2>&1; echo "v20 rc=$?"; grep shape $out/wino_v20.log | python -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['shape'], {k:v['ms'] for k,v in r.items() if k!='shape'})"
timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6 --graph-cells > $out/harness_amoeba_gc.log 2>&1 || { tail -20 $out/harness_amoeba_gc.log; exit 1; }
cat $out/harness_amoeba_gc.log | grep stage
timeout -k 10 600 python -u bench.py --gpus 1 --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 200 python -X faulthandler -u scripts/debug/capture_streams.py --mode step --streams 3 --chunks 1 --steps 2 > $out/step3_m1.log 2>&1; echo "step3_m1 rc=$?"; tail -5 $out/step3_m1.log
