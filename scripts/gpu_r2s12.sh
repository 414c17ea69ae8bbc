# Two-stream AmoebaNet cells (eager and hipGraph-captured): parity tests, then benches.
set -o pipefail
mkdir -p gpurun_out/s12
timeout -k 10 400 python -u -m pytest tests/test_step_graph.py -q --timeout 300 --timeout-method thread > gpurun_out/s12/tests.log 2>&1
rc=$?; tail -3 gpurun_out/s12/tests.log; [ $rc -eq 0 ] || { grep -E "^E " gpurun_out/s12/tests.log | head -30; }
for v in "--cell-streams" "--cell-streams --graph" "--graph"; do
  tag=$(echo "$v" | tr -d ' -')
  timeout -k 10 300 python bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 $v > gpurun_out/s12/amoeba_$tag.log 2>&1 || { tail -20 gpurun_out/s12/amoeba_$tag.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/s12/amoeba_$tag.log | cut -c1-200)"
done
