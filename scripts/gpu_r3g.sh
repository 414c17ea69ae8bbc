# Round 3 call f: batched-GEMM Winograd (4/8-wave tiles, F(4x4) and F(2x2)) numerics + sweep.
set -o pipefail
out=gpurun_out/r3g
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/ops/test_winograd_gpu.py -m gpu -x -q -k "batched" --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $out/tests.log | head -30; exit 1; }
timeout -k 10 600 python -u benchmarks/bg_bench.py --out $out/bg_bench.json > $out/bg_bench.log 2>&1 || { tail -20 $out/bg_bench.log; exit 1; }
python3 - <<'PY'
import json
for r in json.load(open('gpurun_out/r3g/bg_bench.json')):
    print(r['shape'], 'cur', r['current_ms'], 'f4auto', r['f4_auto'], 'f4best', r['f4_best'], r[r['f4_best']], 'f2auto', r['f2_auto'], 'f2best', r['f2_best'], r[r['f2_best']])
PY
