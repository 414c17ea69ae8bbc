# AmoebaNet n1m32 engine options on the final tree (bench.py --model amoebanet): shipped auto
# vs recompute lane / forward overlap (captured cells) and eager cells + weight-gradient stream.
set -o pipefail
out=gpurun_out/r4ar
mkdir -p $out
i=0
for opts in "" "--overlap-recompute on" "--overlap-forward on" "--overlap-recompute on --overlap-forward on" "--graph-cells off --wgrad-stream on" ""; do
  i=$((i+1))
  timeout -k 10 600 python -u bench.py --model amoebanet --sections none $opts > $out/run$i.log 2>&1 || { tail -20 $out/run$i.log; exit 1; }
  echo "run$i [$opts] $(tail -1 $out/run$i.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());c=d["config"];print(d["value"], {k:c.get(k) for k in ("overlap_recompute","wgrad_stream","overlap_forward","cell_streams","graph_cells")})')"
done
