set -o pipefail
mkdir -p gpurun_out/cli
for spec in "unet_speed baseline 4000" "unet_speed pipeline-1 4000" "resnet101_speed baseline 4000" "resnet101_speed pipeline-1 4000"; do
  set -- $spec
  timeout -k 10 300 python benchmarks/$1.py $2 -e 3 -k 1 --dataset-size $3 --json > gpurun_out/cli/$1_$2.log 2>&1 || { tail -5 gpurun_out/cli/$1_$2.log; exit 1; }
  tail -1 gpurun_out/cli/$1_$2.log | cut -c1-250
done
