set -o pipefail
timeout -k 10 200 python benchmarks/wino_variants.py --variants 2 14 15 --shape 40 2048 2048 6 --shape 40 2048 1024 6 --shape 16 2048 2048 6 --shape 16 2048 1024 6 --shape 40 1024 2048 6 > gpurun_out/fwd6.log 2>&1 || exit 1
timeout -k 10 200 python benchmarks/wgrad_variants.py --all-f4 --shape 40 2048 2048 6 --shape 40 2048 1024 6 --shape 16 2048 2048 6 --shape 16 1024 2048 6 > gpurun_out/wg6.log 2>&1 || exit 1
