#!/bin/bash
# r5ay: AmoebaNet n1m32 bench vs the pre-split budget (0 / 2048 / 4096 MiB): does the whole
# 118 M-parameter model's split planes fit the default?
export TMPDIR=/tmp
out=gpurun_out/r5ay
mkdir -p $out
for mb in 2048 4096 0 2048; do
  TGPIPE_CG_PRESPLIT_MB=$mb timeout -k 10 400 python3 bench.py --gpus 1 --model amoebanet --steps 5 --warmup 3 --sections none > $out/n1_$mb.json 2> $out/n1_$mb.err || { tail -20 $out/n1_$mb.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/n1_$mb.json'));print('n1m32 presplit_mb=$mb', d['value'], d['ms_per_step'])"
done
python3 - <<'PY' > $out/budget.log 2>&1
import torch
from torchgpipe_amd.models import amoebanetd
from torchgpipe_amd.ops import _ext
_ext.require()
m = amoebanetd(num_classes=1000, num_layers=18, num_filters=256).cuda().train()
x = torch.rand(20, 3, 224, 224, device='cuda')
torch.ops.tgpipe.conv_gemm_presplit(1 << 20, True)  # no limit
m(x).sum().backward()
torch.cuda.synchronize()
print('presplit bytes held, one fwd+bwd, no limit:', torch.ops.tgpipe.conv_gemm_presplit(-1, True) / 2**20, 'MiB')
PY
cat $out/budget.log | tail -2
