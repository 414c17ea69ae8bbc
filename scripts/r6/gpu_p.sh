#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r6p
t=tests/test_overlap_recompute.py
timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu "$t::test_batchnorm_stage_on_lanes_matches_one_stream" > gpurun_out/r6p/alone.log 2>&1; echo "alone rc=$?"; tail -3 gpurun_out/r6p/alone.log
timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu "$t::test_weight_gradient_stream_matches_plain" "$t::test_batchnorm_stage_on_lanes_matches_one_stream" > gpurun_out/r6p/after_wgrad.log 2>&1; echo "after wgrad rc=$?"; tail -3 gpurun_out/r6p/after_wgrad.log
timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu "$t::test_overlap_with_two_stream_cells_matches_plain" "$t::test_batchnorm_stage_on_lanes_matches_one_stream" > gpurun_out/r6p/after_cells.log 2>&1; echo "after cells rc=$?"; tail -3 gpurun_out/r6p/after_cells.log
