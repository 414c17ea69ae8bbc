set -o pipefail
mkdir -p gpurun_out/r2aj
timeout -k 10 600 python -u -m pytest tests/ops/test_winograd_gpu.py -x -q -k "f4_forward" --timeout 120 --timeout-method thread > gpurun_out/r2aj/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2aj/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/wino_variants.py --variants 6 18 --iters 30 --shape 40 64 64 192 --shape 40 128 64 192 --shape 40 128 128 96 --shape 40 256 128 96 --shape 40 256 256 48 --shape 40 512 256 48 --shape 16 64 64 192 --shape 16 256 256 48 > gpurun_out/r2aj/wino.log 2>&1 || { tail gpurun_out/r2aj/wino.log; exit 1; }
grep shape gpurun_out/r2aj/wino.log | python3 -c "
import sys, json
for l in sys.stdin:
    r=json.loads(l); print(r['shape'], {k:(v['ms'], '%.1e'%v['rel_err']) for k,v in r.items() if k!='shape'})"
