set -o pipefail
mkdir -p gpurun_out/r2q
timeout -k 10 300 python -u benchmarks/convgemm_sweep.py --out gpurun_out/r2q/sweep.json > gpurun_out/r2q/sweep.log 2>&1 || { tail gpurun_out/r2q/sweep.log; exit 1; }
cat gpurun_out/r2q/sweep.log | cut -c1-400
