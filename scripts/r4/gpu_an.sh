# A/B: the 8-wave 128x128 tile interleaving its loads for the plain 1x1 backward-data too
# (variants/_C_bwdint.so; 36 bytes/lane of scratch) vs the shipped build (variants/_C_base.so).
set -o pipefail
out=gpurun_out/r4an
mkdir -p $out
for v in bwdint base; do
  cp variants/_C_$v.so torchgpipe_amd/_C.so
  timeout -k 10 600 python -u benchmarks/convgemm_sweep.py --micro-batch 40 --out $out/sweep_$v.json > $out/sweep_$v.log 2>&1 || { tail -20 $out/sweep_$v.log; exit 1; }
  timeout -k 10 600 python -u bench.py --model resnet --sections none > $out/resnet_$v.log 2>&1 || { tail -20 $out/resnet_$v.log; exit 1; }
  echo "== $v"; tail -1 $out/resnet_$v.log | cut -c1-200
done
