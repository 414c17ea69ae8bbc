# Round 3 final check, then the tuned U-Net balances' stage times.
set -o pipefail
bash scripts/gpu_r3an.sh || exit 1
bash scripts/gpu_r3ap.sh
