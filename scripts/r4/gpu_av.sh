# Kernel trace of ResNet-101 pipeline-1 (B 220, m 2, recompute lane) on the final tree,
# summarised on the box (scripts/r4/rocpd_summary.py) for profiles/r4/rocprof/.
set -o pipefail
out=gpurun_out/r4av
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_resnet_p1 -o run -- python3 bench.py --model resnet --gpus 1 --steps 3 --warmup 3 --sections none > $out/resnet_p1.json 2> $out/resnet_p1.err || { tail -20 $out/resnet_p1.err; exit 1; }
python3 scripts/r4/rocpd_summary.py $out/prof_resnet_p1/run_results.db --last-ms 445 --steps 3 --top 30 > $out/resnet_p1_summary.md && rm -rf $out/prof_resnet_p1
head -12 $out/resnet_p1_summary.md
