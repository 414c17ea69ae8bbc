#!/bin/bash
# One short bench per MIOpen configuration (solver families / find mode); JSON lines
# to gpurun_out/miopen_sweep/.  Usage: bash scripts/miopen_env_sweep.sh
set -o pipefail
out=gpurun_out/miopen_sweep
mkdir -p $out
run() {  # name, env assignments...
  local name=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $out/$name.json 2> $out/$name.err || { echo "$name failed rc=$?"; return 1; }
  echo "$name: $(python -c "import json,sys; d=json.load(open('$out/$name.json')); print(d['value'], d['ms_per_step'], d['config']['warmup_s'])")"
}
run base MIOPEN_LOG_LEVEL=3 && \
run no_winograd MIOPEN_DEBUG_CONV_WINOGRAD=0 && \
run find_normal MIOPEN_FIND_MODE=1 && \
run no_wino_no_direct MIOPEN_DEBUG_CONV_WINOGRAD=0 MIOPEN_DEBUG_CONV_DIRECT=0
