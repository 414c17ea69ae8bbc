# Round 3 call o: the full AmoebaNet two-stream capture crashed inside graph.replay()
# (hipGraphLaunch).  Hypothesis: the runtime walks the (multi-stream, ~100k-node) DAG
# recursively and overflows the 8 MiB main-thread stack.  Same run with an unlimited stack.
set -o pipefail
out=gpurun_out/r3o
mkdir -p $out
export TGPIPE_CAPTURE_STREAMS=1
ulimit -s unlimited
echo "stack: $(ulimit -s)"
timeout -k 10 400 python -X faulthandler bench.py --model amoebanet --graph --cell-streams on --steps 3 --warmup 3 --sections none > $out/full.json 2> $out/full.err
rc=$?; echo "full rc=$rc"; grep -v "Cannot find the function" $out/full.err | tail -30 | cut -c1-200; cat $out/full.json | cut -c1-300
exit 0
