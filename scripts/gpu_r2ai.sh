set -o pipefail
rm -rf gpurun_out/pmc4r2
OP=fwd4 bash scripts/pmc_wino.sh gpurun_out/pmc4r2 "40 64 64 192" "40 128 128 96" "40 256 256 48" || exit 1
OP=wgrad4 bash scripts/pmc_wino.sh gpurun_out/pmc4r2 "40 64 64 192" "40 256 256 48" || exit 1
for f in gpurun_out/pmc4r2/p1_*/run_counter_collection.csv; do python3 scripts/pmc_table.py $f --kernel f4_ ; done > gpurun_out/pmc4r2/table.txt
echo DONE
