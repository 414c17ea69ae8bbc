# rocprofv3 kernel trace of a bench.py run, summarised on the box (the raw database
# is deleted: it is too large to copy back).  Usage: bash scripts/profile_bench.sh <tag> [bench args]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/prof_$tag
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_$tag -o run -- python3 bench.py "$@" > gpurun_out/prof_$tag/bench.log 2>&1 || exit 1
db=$(find gpurun_out/prof_$tag -name '*.db' | head -1)
python3 scripts/rocpd_summary.py "$db" --skip 2 --csv gpurun_out/prof_$tag/kernel_stats.csv \
    --md gpurun_out/prof_$tag/summary.md --title "$tag" > /dev/null || exit 1
rm -f "$db"
