# Kernel traces of the final tree: U-Net(5,64) pipeline-1 (the headline) and AmoebaNet n1m32
# (captured three-stream cells), summarised on the box (scripts/r4/rocpd_summary.py) for
# profiles/r4/rocprof/; the databases themselves are deleted (too large to bring back).
set -o pipefail
out=gpurun_out/r4ah
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_unet_p1 -o run -- python3 bench.py --gpus 1 --steps 3 --warmup 3 --sections none > $out/unet_p1.json 2> $out/unet_p1.err || { tail -20 $out/unet_p1.err; exit 1; }
python3 scripts/r4/rocpd_summary.py $out/prof_unet_p1/run_results.db --last-ms 370 --steps 3 --top 30 > $out/unet_p1_summary.md && rm -rf $out/prof_unet_p1
head -3 $out/unet_p1_summary.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_amoeba_n1 -o run -- python3 bench.py --model amoebanet --gpus 1 --steps 2 --warmup 4 --sections none > $out/amoeba_n1.json 2> $out/amoeba_n1.err || { tail -20 $out/amoeba_n1.err; exit 1; }
python3 scripts/r4/rocpd_summary.py $out/prof_amoeba_n1/run_results.db --last-ms 3420 --steps 2 --top 30 > $out/amoeba_n1_summary.md && rm -rf $out/prof_amoeba_n1
head -3 $out/amoeba_n1_summary.md
