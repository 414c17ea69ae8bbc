set -o pipefail
mkdir -p gpurun_out/r2al
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/skip/test_gpipe.py -x -q -s -k "fused_unet_matches or 1to3" --timeout 120 --timeout-method thread > gpurun_out/r2al/tests.log 2>&1
rc=$?; grep -E "relative gradient|passed|failed|Error" gpurun_out/r2al/tests.log | cut -c1-3000; exit $rc
