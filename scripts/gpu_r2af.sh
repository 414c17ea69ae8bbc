set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/profile_bench.sh unet_r2af --gpus 1 --steps 4 --warmup 2 || exit 1
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_unet_r2af/kernel_stats.csv')))
for r in rows[:45]:
    print('%6d calls/step %7.2f ms/step  %s'%(int(r['Calls'])/4, int(r['TotalDurationNs'])/4e6, r['Name'][:100]))
PY
