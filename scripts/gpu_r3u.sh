# Round 3: diagnose the fused 3x3 (256 channels @ 14^2) Conv-BN-ReLU x.grad mismatch.
set -o pipefail
out=gpurun_out/r3u
mkdir -p $out
PYTHONPATH=. timeout -k 10 200 python benchmarks/diag/resnet_fused_diag.py 2>&1 | tee $out/diag.log
TGPIPE_BN_BWD_ONEPASS=0 PYTHONPATH=. timeout -k 10 200 python benchmarks/diag/resnet_fused_diag.py 2>&1 | tee $out/diag_twopass.log
TGPIPE_WINOGRAD_BG=0 PYTHONPATH=. timeout -k 10 200 python benchmarks/diag/resnet_fused_diag.py 2>&1 | tee $out/diag_nobg.log
