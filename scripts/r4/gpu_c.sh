set -o pipefail
out=gpurun_out/r4c
mkdir -p $out
timeout -k 10 300 python -u scripts/debug/seg_parity.py > $out/seg_parity.log 2>&1; rc=$?
cat $out/seg_parity.log | tail -40
exit $rc
