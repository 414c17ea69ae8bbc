# AmoebaNet n1m32 on one GPU: whole-step hipGraph (two-stream cells, bench default) vs
# captured cells (three-stream cells), each twice.
set -o pipefail
out=gpurun_out/r4y
mkdir -p $out
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --model amoebanet --gpus 1 --steps 10 --warmup 3 --sections none > $out/step_$rep.json 2> $out/step_$rep.err || { tail -20 $out/step_$rep.err; exit 1; }
  timeout -k 10 300 python -u bench.py --model amoebanet --gpus 1 --steps 10 --warmup 4 --sections none --graph-cells on > $out/cells_$rep.json 2> $out/cells_$rep.err || { tail -20 $out/cells_$rep.err; exit 1; }
  python -c "import json;a=json.load(open('$out/step_$rep.json'));b=json.load(open('$out/cells_$rep.json'));print('step graph', a['value'], a['config']['cell_streams'], '| cells', b['value'], b['config']['cell_streams'])"
done
