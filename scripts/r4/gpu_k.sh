# AmoebaNet implicit-GEMM shapes at micro-batch 40 (the n*m32 experiments): per-shape table vs
# MIOpen, every launch plan of the sweep shapes, PMC of the 7x7 / 14x14 GEMMs.
set -o pipefail
out=gpurun_out/r4k
mkdir -p $out
timeout -k 10 300 python -u benchmarks/diag/resnet_strided_probe.py > $out/resnet_strided_probe.jsonl 2> $out/resnet_strided_probe.err || { tail -20 $out/resnet_strided_probe.err; exit 1; }
python -c "
import json
for l in open('$out/resnet_strided_probe.jsonl'):
    r=json.loads(l); print(r['name'], 'miopen dgrad', r['bwd_data_us'], 'native', r.get('native_bwd_data_us'), '| conv+bn miopen', r['miopen_bn_fwd_bwd_us'], 'fused', r.get('fused_fwd_bwd_us'), 'fused native', r.get('fused_native_fwd_bwd_us'))"
timeout -k 10 300 python -u benchmarks/convbn_bench.py --micro-batch 40 --out $out/convbn_bench_n40.json > $out/convbn_bench.log 2>&1 || { tail -20 $out/convbn_bench.log; exit 1; }
tail -1 $out/convbn_bench.log
timeout -k 10 300 python -u benchmarks/convgemm_sweep.py --micro-batch 40 --out $out/convgemm_sweep_n40.json > $out/sweep.log 2>&1 || { tail -20 $out/sweep.log; exit 1; }
export TMPDIR=/tmp
for spec in "fwd 1024 7 1024 1 1" "bwd 1024 7 1024 1 1" "wgrad 1024 7 1024 1 1" "fwd 4096 7 1024 1 1" "fwd 512 14 512 1 1" "wgrad 512 14 512 1 1"; do
  set -- $spec; tag=$1_$2_$3_$4_$5x$6
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/pmc/$tag -o run -- python3 benchmarks/convgemm_probe.py --x 40 $2 $3 $3 --co $4 --k $5 $6 --mode $1 --iters 10 > $out/pmc_$tag.log 2>&1 || { tail $out/pmc_$tag.log; exit 1; }
done
echo DONE
