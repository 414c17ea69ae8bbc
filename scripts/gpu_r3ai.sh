# Round 3: 1x1 convolutions as library GEMMs vs the implicit-GEMM kernels (ResNet / AmoebaNet shapes).
set -o pipefail
out=gpurun_out/r3ai
mkdir -p $out
PYTHONPATH=. timeout -k 10 300 python benchmarks/diag/gemm_lib_probe.py > $out/gemm_lib_probe.jsonl 2> $out/gemm_lib_probe.err || { tail -20 $out/gemm_lib_probe.err; exit 1; }
cat $out/gemm_lib_probe.jsonl
