# Stride-2 1x1 backward-data fill with the grid.z phase order restored: GPU suite,
# micro-batch-40 per-shape table, default one-GPU bench.
set -o pipefail
out=gpurun_out/r4al
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 600 python -u benchmarks/convbn_bench.py --micro-batch 40 --out $out/convbn_bench_n40.json > $out/convbn.log 2>&1 || { tail -20 $out/convbn.log; exit 1; }
tail -1 $out/convbn.log
timeout -k 10 900 python -u bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log
