set -o pipefail
OP=fwd4 bash scripts/pmc_wino.sh gpurun_out/pmc4 "40 256 256 48" "40 64 64 192" || exit 1
OP=wgrad4 bash scripts/pmc_wino.sh gpurun_out/pmc4 "40 256 256 48" || exit 1
echo DONE
