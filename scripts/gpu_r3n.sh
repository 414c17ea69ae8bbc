# Round 3 call n: root-cause the multi-stream hipGraph capture crash of the full AmoebaNet
# step (profiles/r2/bench_amoeba_n1m32_s13_streams_graph_crash.log): tiny model first, then
# the full one, both with two-stream cells allowed inside the capture, faulthandler on.
set -o pipefail
out=gpurun_out/r3n
mkdir -p $out
export TGPIPE_CAPTURE_STREAMS=1 AMD_LOG_LEVEL=1
timeout -k 10 300 python -X faulthandler bench.py --model amoebanet --tiny --batch 8 --chunks 4 --graph --cell-streams on --steps 3 --warmup 3 --sections none > $out/tiny.json 2> $out/tiny.err
echo "tiny rc=$?"; tail -3 $out/tiny.err
timeout -k 10 400 python -X faulthandler bench.py --model amoebanet --graph --cell-streams on --steps 3 --warmup 3 --sections none > $out/full.json 2> $out/full.err
rc=$?; echo "full rc=$rc"; tail -60 $out/full.err | cut -c1-200
exit 0
