# Debug probe: weight-gradient stream over several SGD steps.
set -o pipefail
mkdir -p gpurun_out/s20
timeout -k 10 400 python scripts/debug/wgrad_stream_steps.py > gpurun_out/s20/steps.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/s20/steps.log | grep -v Warning | tail -8; exit $rc
