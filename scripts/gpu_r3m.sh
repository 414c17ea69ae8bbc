# Round 3 call k: vectorised input transform, tuned tiles; sweep incl. shallow levels; p1 bench.
set -o pipefail
out=gpurun_out/r3m
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/ops/test_winograd_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $out/tests.log | head -30; exit 1; }
timeout -k 10 600 python -u benchmarks/bg_bench.py --out $out/bg_bench.json > $out/bg_bench.log 2>&1 || { tail -20 $out/bg_bench.log; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --sections none > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print('p1', d['value'], d['ms_per_step'])"
python3 - <<'PY'
import json
for r in json.load(open('gpurun_out/r3m/bg_bench.json')):
    ks=[k for k in r if k[:4] in ('f4_4','f4_1','f2_4','f2_1')]
    print(r['shape'], 'cur', r['current_ms'], 'f4auto', r['f4_auto'], ' '.join(f"{k[:2]}{k[4:]}={r[k]}" for k in ks))
PY
