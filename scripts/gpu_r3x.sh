# Round 3: r3v + r3w in one call (the pool is congested).
set -o pipefail

bash scripts/gpu_r3v.sh || exit 1
