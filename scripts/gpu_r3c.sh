# Round 3 call c: per-kernel stats (csv) of the heaviest reference-balance stages and a
# cProfile of the host side of p8 stage 3.
set -o pipefail
out=gpurun_out/r3c
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p8s3 -o run -- python3 benchmarks/stage_harness.py --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 --stages 3 > $out/p8s3.log 2>&1 || { tail -5 $out/p8s3.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/p4s2 -o run -- python3 benchmarks/stage_harness.py --model unet --balance 30 66 84 61 --chunks 16 --batch 512 --stages 2 > $out/p4s2.log 2>&1 || { tail -5 $out/p4s2.log; exit 1; }
find $out -name '*kernel_trace.csv' -delete
find $out -name '*stats.csv'
timeout -k 10 300 python3 -m cProfile -o $out/p8s3.prof benchmarks/stage_harness.py --model unet --balance 16 27 31 44 22 57 27 17 --chunks 40 --batch 640 --stages 3 > $out/p8s3_cprof.log 2>&1 || { tail -5 $out/p8s3_cprof.log; exit 1; }
python3 -c "
import pstats; s=pstats.Stats('$out/p8s3.prof'); s.sort_stats('tottime').print_stats(45)" > $out/p8s3_prof_tottime.txt
python3 -c "
import pstats; s=pstats.Stats('$out/p8s3.prof'); s.sort_stats('cumulative').print_stats(60)" > $out/p8s3_prof_cum.txt
tail -1 $out/p8s3_cprof.log
