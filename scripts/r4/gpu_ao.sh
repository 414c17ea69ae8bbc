# Weight-gradient loads over planes of 4k+r pixels with one division per quad (the image
# advances at most once): GPU suite, sweep / per-shape table at micro-batch 40, bench.
set -o pipefail
out=gpurun_out/r4ao
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -40 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 600 python -u benchmarks/convgemm_sweep.py --micro-batch 40 --out $out/sweep.json > $out/sweep.log 2>&1 || { tail -20 $out/sweep.log; exit 1; }
timeout -k 10 600 python -u benchmarks/convbn_bench.py --micro-batch 40 --out $out/convbn_bench_n40_wt.json > $out/convbn.log 2>&1 || { tail -20 $out/convbn.log; exit 1; }
tail -1 $out/convbn.log
timeout -k 10 900 python -u bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-160
python -c "import json;d=json.loads(open('$out/bench.log').read().strip().splitlines()[-1]);print('unet', d['value'], 'base', d['baseline']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'])"
