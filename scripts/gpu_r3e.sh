# Round 3 call e: batched-GEMM F(2x2) numerics, per-kernel times and PMC of bg_conv.
set -o pipefail
out=gpurun_out/r3e
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/ops/test_winograd_gpu.py -m gpu -x -q -k "batched" --timeout 120 --timeout-method thread > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $out/tests.log | head -30; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for spec in "16 1024 1024 12 4" "32 512 512 24 4" "16 2048 2048 6 4" "16 2048 2048 6 2" "40 2048 2048 6 2"; do
  set -- $spec; tag=s$1_$2_$3_$4_k$5
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$tag -o run -- python3 benchmarks/bg_probe.py --shape $1 $2 $3 $4 --kind $5 --iters 10 > $out/$tag.log 2>&1 || { tail -3 $out/$tag.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_$tag -o run -- python3 benchmarks/bg_probe.py --shape $1 $2 $3 $4 --kind $5 --iters 5 > $out/pmc_$tag.log 2>&1 || { tail -3 $out/pmc_$tag.log; exit 1; }
done
find $out -name '*kernel_trace.csv' -path '*/s*' -delete
echo DONE
