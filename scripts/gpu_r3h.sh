# Round 3 call h: batched-GEMM dispatch end to end: GPU tests, bench, reference-balance stages.
set -o pipefail
out=gpurun_out/r3h
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -2 $out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $out/gpu_tests.log | head -30; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --sections baseline > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print('p1', d['value'], d['ms_per_step'], 'baseline', d['baseline_samples_per_sec'], 'speedup', d['speedup_vs_baseline'])"
timeout -k 10 300 python benchmarks/stage_harness.py --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 --out $out/stage_p8.json > $out/stage_p8.log 2>&1 || { tail -5 $out/stage_p8.log; exit 1; }
timeout -k 10 300 python benchmarks/stage_harness.py --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --out $out/stage_p4.json > $out/stage_p4.log 2>&1 || { tail -5 $out/stage_p4.log; exit 1; }
timeout -k 10 300 python benchmarks/stage_harness.py --model unet --balance 104 137 --chunks 32 --batch 512 --out $out/stage_p2.json > $out/stage_p2.log 2>&1 || { tail -5 $out/stage_p2.log; exit 1; }
cat $out/stage_p8.log $out/stage_p4.log $out/stage_p2.log | grep stage
