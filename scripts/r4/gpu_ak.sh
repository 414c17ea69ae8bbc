# Stride phases as the fastest block index (one tile's phases together on one XCD) and the
# stride-2 1x1 backward-data writing its own hole zeros: the GPU suite, then the
# micro-batch-40 per-shape table with and without the fill.
set -o pipefail
out=gpurun_out/r4ak
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 600 python -u benchmarks/convbn_bench.py --micro-batch 40 --out $out/convbn_bench_n40.json > $out/convbn.log 2>&1 || { tail -20 $out/convbn.log; exit 1; }
tail -1 $out/convbn.log
TGPIPE_CG_FILL=0 timeout -k 10 600 python -u benchmarks/convbn_bench.py --micro-batch 40 --out $out/convbn_bench_n40_nofill.json > $out/convbn_nofill.log 2>&1 || { tail -20 $out/convbn_nofill.log; exit 1; }
tail -1 $out/convbn_nofill.log
