# First-step diagnosis (plan misses) and the 6x6 bottleneck convolutions at micro-batch 40:
# F(2x2) / F(4x4) variants x split counts.
set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 200 python benchmarks/first_step.py --model amoebanet --top 25 > gpurun_out/s4/first_amoeba.log 2>&1 || { tail -20 gpurun_out/s4/first_amoeba.log; exit 1; }
grep -E "^(build|step|plans)" gpurun_out/s4/first_amoeba.log
timeout -k 10 300 python benchmarks/wino_variants.py --variants 0 1 2 14 15 --splits 0 1 2 3 4 6 8 --iters 10 --shape 40 1024 2048 6 --shape 40 2048 2048 6 --shape 40 2048 1024 6 --out gpurun_out/s4/wino_6x6_mb40.json > gpurun_out/s4/wino.log 2>&1 || { tail -20 gpurun_out/s4/wino.log; exit 1; }
python - <<'PY'
import json
for r in json.load(open('gpurun_out/s4/wino_6x6_mb40.json')):
    best = sorted(((v['ms'], k, v['rel_err']) for k, v in r.items() if k != 'shape'))[:6]
    print(r['shape'], [(k, ms, f'{e:.1e}') for ms, k, e in best], 'auto:', {k: r[k]['ms'] for k in ('v0', 'v2', 'v14', 'v15')})
PY
