# ResNet-101 pipeline-1 engine variants (plain stage, recompute lane, captured cells, the
# single-process GPipe engine of benchmarks/diag), a kernel profile of the slowest
# AmoebaNet n8m32 stage with captured cells, and the U-Net(48,160) p8 memory benchmark.
set -o pipefail
out=gpurun_out/r4i
mkdir -p $out
r() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --model resnet --gpus 1 --steps 10 --warmup 3 --sections none "$@" > $out/$name.json 2> $out/$name.err || { echo "$name failed"; tail -20 $out/$name.err; return 1; }
  python -c "import json;d=json.load(open('$out/$name.json'));print('$name', d['value'], d['ms_per_step'], d['config']['rank0_peak_mem_gib'])"
}
r resnet_plain || exit 1
r resnet_lanes --overlap-recompute on || exit 1
r resnet_gc --graph-cells on --warmup 4 || exit 1
r resnet_gc_lanes --graph-cells on --overlap-recompute on --warmup 4 || exit 1
timeout -k 10 300 python -u benchmarks/diag/resnet_kernel_table.py --rows 25 > $out/resnet_gpipe_table.txt 2>&1 || { tail -20 $out/resnet_gpipe_table.txt; exit 1; }
head -3 $out/resnet_gpipe_table.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_amoeba_s6 -o run -- python3 benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 6 --graph-cells --steps 2 > $out/prof_amoeba_s6.log 2>&1 || { tail -20 $out/prof_amoeba_s6.log; exit 1; }
grep '"stage"' $out/prof_amoeba_s6.log
timeout -k 10 1200 python -u benchmarks/memory.py unet --experiment pipeline-8 --out $out/memory_unet_48_160_p8.json > $out/memory.log 2>&1 || { tail -20 $out/memory.log; exit 1; }
tail -12 $out/memory.log
