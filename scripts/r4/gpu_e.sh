# Three-stream capture investigation (ADVICE / Next #5): per-cell graphs vs whole-step
# graph, DAG-size dependence, and the HIP API call in progress at the crash.
set -o pipefail
out=gpurun_out/r4e
mkdir -p $out
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python -X faulthandler -u scripts/debug/capture_streams.py "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 $out/$name.log
  return $rc
}
run cells3_m32 300 --mode cells --streams 3 --chunks 32 --steps 3 || exit 1
run step3_m4 300 --mode step --streams 3 --chunks 4 --steps 2 || exit 1
run step3_m12 300 --mode step --streams 3 --chunks 12 --steps 2 || exit 1
# the full step: expected to crash; keep the last HIP API log lines
AMD_LOG_LEVEL=3 timeout -k 10 400 python -X faulthandler -u scripts/debug/capture_streams.py --mode step --streams 3 --chunks 32 --steps 2 > $out/step3_m32.log 2> >(tail -c 400000 > $out/step3_m32.err)
echo "== step3_m32 rc=$?"; tail -4 $out/step3_m32.log; sleep 2; tail -30 $out/step3_m32.err
