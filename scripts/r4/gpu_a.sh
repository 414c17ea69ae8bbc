# Round 4 first check: GPU suite after the housekeeping commit, smoke.
set -o pipefail
out=gpurun_out/r4a
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1; rc=$?
tail -15 $out/gpu_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
