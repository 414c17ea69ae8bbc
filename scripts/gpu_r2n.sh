set -o pipefail
mkdir -p gpurun_out/r2n
timeout -k 10 300 python -u benchmarks/wino_variants.py --variants 6 16 17 --iters 30 --shape 40 64 64 192 --shape 40 128 64 192 --shape 40 128 128 96 --shape 40 256 128 96 --shape 40 256 256 48 --shape 40 512 256 48 --shape 16 64 64 192 --shape 16 128 128 96 --shape 16 256 256 48 --shape 3 70 130 13 --shape 2 8 8 20 --out gpurun_out/r2n/wino.json > gpurun_out/r2n/wino.log 2>&1 || { tail gpurun_out/r2n/wino.log; exit 1; }
cat gpurun_out/r2n/wino.log
