# Round 3, first GPU call: full GPU test suite (incl. shared-GPU multi-rank rehearsals
# with lanes / two-stream cells), smoke, default bench (U-Net p1 + baseline + AmoebaNet).
set -o pipefail
out=gpurun_out/r3a
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 120 python __graft_entry__.py smoke > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cut -c1-400 $out/bench.json
grep -c "AccumulateGrad" $out/bench.err || true
