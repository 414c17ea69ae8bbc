#!/bin/bash
# r5ao: bisect the whole-step StepGraph replay mismatch: pre-split weights off / fused
# small-plane split BatchNorm off / both on
export TMPDIR=/tmp
out=gpurun_out/r5ao
mkdir -p $out
t() { name=$1; shift; env "$@" timeout -k 10 300 python -u -m pytest tests/test_step_graph.py -m gpu -q --timeout 200 --timeout-method thread > $out/$name.log 2>&1; echo "$name rc=$? $(tail -1 $out/$name.log)"; }
t default TGPIPE_X=1
t presplit_off TGPIPE_CG_PRESPLIT_MB=0
t splitbn_off TGPIPE_SPLIT_BN=0
