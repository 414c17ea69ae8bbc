# AmoebaNet n8m32 stage 6's layers one at a time (reduction cell 16, normal cells 17-19) at
# micro-batch 40, and a kernel trace of the reduction cell alone.
set -o pipefail
out=gpurun_out/r4v
mkdir -p $out
timeout -k 10 300 python -u benchmarks/stage_harness.py --model amoebanet --balance 16 1 1 1 1 4 --chunks 32 --batch 1280 --stages 1 2 3 4 --graph-cells --out $out/layers_16_19.json > $out/layers.log 2>&1 || { tail -20 $out/layers.log; exit 1; }
grep '"stage"' $out/layers.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_l16 -o run -- python3 benchmarks/stage_harness.py --model amoebanet --balance 16 1 7 --chunks 32 --batch 1280 --stages 1 --graph-cells --steps 2 > $out/prof_l16.log 2>&1 || { tail -20 $out/prof_l16.log; exit 1; }
grep '"stage"' $out/prof_l16.log
