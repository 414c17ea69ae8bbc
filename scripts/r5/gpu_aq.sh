#!/bin/bash
# r5aq: pre-split weights with captured cells: a weight missing from the cache inside a
# capture keeps the in-kernel split (no derive node per replay); GPU numerics of the fused
# ops / graphs / segments, then the AmoebaNet n1m32 bench headline under rocprof
export TMPDIR=/tmp
out=gpurun_out/r5aq
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/ops/test_convbn_gpu.py tests/ops/test_group_convbn_gpu.py tests/test_step_graph.py tests/test_segments.py tests/models -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
summ() {  # dir steps ms_per_step name
  python3 scripts/r4/rocpd_summary.py $1/run_results.db --last-ms $3 --steps $2 --top 40 > $out/$4.md && rm -rf $1
  head -3 $out/$4.md; grep -n "presplit\|elementwise_kernel_manual" $out/$4.md || true
}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/p_amoeba -o run -- python3 bench.py --gpus 1 --model amoebanet --steps 2 --warmup 3 --sections none > $out/amoeba_n1.json 2> $out/amoeba_n1.err || { tail -20 $out/amoeba_n1.err; exit 1; }
ms=$(python3 -c "import json;d=json.load(open('$out/amoeba_n1.json'));print(d['ms_per_step']*2)")
summ $out/p_amoeba 2 $ms amoeba_n1m32
timeout -k 10 400 python3 bench.py --gpus 1 --model amoebanet --steps 5 --warmup 3 --sections none > $out/amoeba_n1_bench.json 2> $out/amoeba_n1_bench.err || { tail -20 $out/amoeba_n1_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$out/amoeba_n1_bench.json'));print('n1m32', d['value'], d['ms_per_step'])"
