set -o pipefail
timeout -k 10 300 python -u -m pytest tests/ops/test_winograd_gpu.py -x -q --timeout 120 --timeout-method thread -k "f4" > gpurun_out/f4_tests.log 2>&1 || { tail -30 gpurun_out/f4_tests.log; exit 1; }
tail -1 gpurun_out/f4_tests.log
timeout -k 10 300 python benchmarks/wino_variants.py --variants 6 7 14 15 --shape 40 64 64 192 --shape 40 256 256 48 --shape 40 1024 1024 12 --shape 16 512 512 24 --shape 40 128 128 96 --shape 40 2048 2048 6 > gpurun_out/abl.log 2>&1 || { tail gpurun_out/abl.log; exit 1; }
echo DONE
