"""AvgPool3x3 forward / backward times (HIP events, median of 20) at AmoebaNet-D(18,256)'s
plane shapes, micro-batch 20 (n1m32) -- scripts/r6/gpu_u.sh."""
import json
import sys

import torch

sys.path.insert(0, '.')
from torchgpipe_amd.ops.pool import AvgPool3x3  # noqa: E402


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(iters):
        a.record()
        fn()
        b.record()
        b.synchronize()
        out.append(a.elapsed_time(b) * 1000)
    return sorted(out)[iters // 2]


for n, c, h, stride in [(20, 64, 56, 1), (20, 128, 56, 2), (20, 128, 28, 1), (20, 256, 28, 2),
                        (20, 256, 14, 1), (20, 512, 14, 2), (40, 128, 28, 1)]:
    x = torch.randn(n, c, h, h, device='cuda', requires_grad=True)
    pool = AvgPool3x3(stride)
    y = pool(x, None)
    g = torch.randn_like(y)
    fwd = timed(lambda: pool(x, None))
    bwd = timed(lambda: torch.autograd.grad(pool(x, None), x, g)) - fwd
    mb = (x.numel() + y.numel()) * 4 / 1e6
    print(json.dumps({'shape': [n, c, h, h], 'stride': stride, 'fwd_us': round(fwd, 1),
                      'bwd_us': round(bwd, 1), 'fwd_GBps': round(mb / fwd * 1e3, 0)}),
          flush=True)
