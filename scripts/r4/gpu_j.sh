# Default bench (sections released between timings, ResNet recompute lane), the GPipe-engine
# ResNet table, ResNet-101 p2 at 110-image micro-batches (stage harness), a kernel profile of
# the slowest AmoebaNet n8m32 stage with captured cells, the U-Net(48,160) p8 memory run.
set -o pipefail
out=gpurun_out/r4j
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/ops/test_convbn_gpu.py -q -x --timeout 120 --timeout-method thread -k "conv_gemm_matches or phases" > $out/conv_tests.log 2>&1 || { tail -30 $out/conv_tests.log; exit 1; }
tail -2 $out/conv_tests.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python -c "import json;d=json.load(open('$out/bench.json'));print('unet', d['value'], 'base', d['baseline']['value'], 'amoeba', d['amoebanet']['value'], 'resnet', d['resnet101']['value'], d['resnet101'].get('baseline',{}).get('value'))"
grep -i "still held" $out/bench.err || true
timeout -k 10 300 python -u benchmarks/diag/resnet_kernel_table.py --rows 25 > $out/resnet_gpipe_table.txt 2>&1 || { tail -20 $out/resnet_gpipe_table.txt; exit 1; }
head -3 $out/resnet_gpipe_table.txt
timeout -k 10 600 python -u benchmarks/stage_harness.py --model resnet101 --balance 135 235 --chunks 32 --batch 3520 --checkpoint always --graph-cells --lanes on --out $out/resnet_p2_mb110.json > $out/resnet_p2_mb110.log 2>&1 || { tail -20 $out/resnet_p2_mb110.log; exit 1; }
grep '"stage"' $out/resnet_p2_mb110.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_amoeba_s6 -o run -- python3 benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 --chunks 32 --batch 1280 --stages 6 --graph-cells --steps 2 > $out/prof_amoeba_s6.log 2>&1 || { tail -20 $out/prof_amoeba_s6.log; exit 1; }
grep '"stage"' $out/prof_amoeba_s6.log
timeout -k 10 1200 python -u benchmarks/memory.py unet --experiment pipeline-8 --out $out/memory_unet_48_160_p8.json > $out/memory.log 2>&1 || { tail -20 $out/memory.log; exit 1; }
tail -12 $out/memory.log
