# Debug probe: two-stream cells vs a one-stream copy with the same parameters, per SGD step.
set -o pipefail
mkdir -p gpurun_out/s21
timeout -k 10 300 python scripts/debug/cell_streams_multistep.py > gpurun_out/s21/probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/s21/probe.log | grep -v -i warn | tail -8; exit $rc
