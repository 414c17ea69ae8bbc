# Every AmoebaNet-D(18,256) layer as its own stage at micro-batch 40 (32 micro-batches,
# captured three-stream cells) on the final tree, for the MI355X balances (bench.py `tuned`).
set -o pipefail
out=gpurun_out/r4af
mkdir -p $out
timeout -k 10 900 python -u benchmarks/stage_harness.py --model amoebanet --balance 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 1 --chunks 32 --batch 1280 --graph-cells --out $out/amoeba_layers_mb40.json > $out/layers.log 2>&1 || { tail -20 $out/layers.log; exit 1; }
grep -c '"stage"' $out/layers.log
