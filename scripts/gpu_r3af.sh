# Round 3: kernel traces of U-Net p4 reference-balance stages 1 and 2 (the two stages above
# the reference's speed-up curve) from benchmarks/stage_harness.py (1 warm-up + 2 timed
# passes of all 16 micro-batches: the summary counts the whole trace as 3 passes).
set -o pipefail
out=gpurun_out/r3af
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for st in 1 2; do
  d=gpurun_out/prof_p4s$st
  mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run -- python3 benchmarks/stage_harness.py --balance 30 66 84 61 --chunks 16 --batch 512 --stages $st > $out/p4s$st.log 2>&1 || { tail -20 $out/p4s$st.log; exit 1; }
  db=$(find $d -name '*.db' | head -1)
  python3 scripts/rocpd_summary.py "$db" --whole 3 --csv $out/p4s${st}_kernel_stats.csv --md $out/p4s${st}_summary.md --title "unet p4 ref stage $st" > /dev/null || exit 1
  rm -f "$db"
  grep stage $out/p4s$st.log
  head -30 $out/p4s${st}_summary.md
done
