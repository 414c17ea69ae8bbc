# AmoebaNet n8m32 stages 5 and 6 with the recompute lane (overlap_recompute) on top of the
# three-stream captured cells.
set -o pipefail
out=gpurun_out/r4ab
mkdir -p $out
timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6 --graph-cells --lanes on > $out/s56_lanes.log 2>&1 || { tail -20 $out/s56_lanes.log; exit 1; }
grep '"stage"' $out/s56_lanes.log
timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 5 6 --graph-cells > $out/s56.log 2>&1 || { tail -20 $out/s56.log; exit 1; }
grep '"stage"' $out/s56.log
