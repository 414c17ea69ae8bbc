# Debug probe: which gradients differ with the weight-gradient stream.
set -o pipefail
mkdir -p gpurun_out/s16
timeout -k 10 300 python scripts/debug/wgrad_stream_probe.py > gpurun_out/s16/probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/s16/probe.log | tail -12; exit $rc
