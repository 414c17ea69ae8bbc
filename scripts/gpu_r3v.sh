# Round 3: ResNet-101 pipeline-1 plain (MIOpen) crash check, kernel traces of the fused
# ResNet-101 pipeline-1 and of AmoebaNet n1m32 (eager), grouped-ConvBN tests.
set -o pipefail
out=gpurun_out/r3v
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
(cd benchmarks && timeout -k 10 300 python -X faulthandler resnet101_speed.py pipeline-1 --plain --epochs 3 --skip-epochs 1 --dataset-size 2200 --json > ../$out/resnet_p1_plain.json 2> ../$out/resnet_p1_plain.err); echo "plain rc=$? $(cat $out/resnet_p1_plain.json)"
tail -5 $out/resnet_p1_plain.err
mkdir -p gpurun_out/prof_resnet
(cd benchmarks && timeout -k 10 400 rocprofv3 --kernel-trace -d ../gpurun_out/prof_resnet -o run -- python3 resnet101_speed.py pipeline-1 --epochs 2 --skip-epochs 1 --dataset-size 1100 > ../gpurun_out/prof_resnet/bench.log 2>&1) || exit 1
db=$(find gpurun_out/prof_resnet -name '*.db' | head -1)
python3 scripts/rocpd_summary.py "$db" --skip 5 --csv gpurun_out/prof_resnet/kernel_stats.csv --md gpurun_out/prof_resnet/summary.md --title resnet101_p1_fused > /dev/null || exit 1
rm -f "$db"
head -40 gpurun_out/prof_resnet/summary.md
bash scripts/profile_bench.sh amoeba_r3v --model amoebanet --graph off --steps 3 --warmup 2 --sections none || exit 1
head -30 gpurun_out/prof_amoeba_r3v/summary.md
