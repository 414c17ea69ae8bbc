# Round 3 call p: graph tests with two-stream captures, default bench (AmoebaNet graphed).
set -o pipefail
out=gpurun_out/r3p
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_step_graph.py tests/test_overlap_recompute.py tests/models -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $out/tests.log | head -30; exit 1; }
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json'))
print('unet p1', d['value'], 'baseline', d['baseline_samples_per_sec'], 'speedup', d['speedup_vs_baseline'])
print('amoeba', d['amoebanet'])"
