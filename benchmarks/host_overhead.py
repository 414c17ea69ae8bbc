"""Host (CPU) cost per call of the U-Net cell ops, on shapes too small to keep the GPU busy.

A pipeline stage is launch-bound when its host enqueue time approaches its device time
(benchmarks/stage_harness.py reports both); this measures where the host time goes.

    python benchmarks/host_overhead.py
"""
import json
import os
import sys
import time

import torch
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torchgpipe_amd.models.unet import conv_block  # noqa: E402
from torchgpipe_amd.ops import _ext  # noqa: E402
from torchgpipe_amd.ops.conv import WinogradConv2d  # noqa: E402
from torchgpipe_amd.ops.fused import DropNormAct  # noqa: E402


def host_us(fn, iters=300):  # type: ignore[no-untyped-def]
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    host = (time.perf_counter() - t) / iters * 1e6
    torch.cuda.synchronize()
    return round(host, 1)


def main() -> None:
    dev = torch.device('cuda')
    ops = _ext.require()
    x = torch.randn(2, 64, 16, 16, device=dev, requires_grad=True)
    conv = WinogradConv2d(64, 64, 3, padding=1).to(dev)
    plain = nn.Conv2d(64, 64, 3, padding=1).to(dev)
    dna = DropNormAct().to(dev)
    cell = conv_block(64, 64, True).to(dev)
    u4 = ops.wino4_weight(conv.weight.detach(), False)
    xd = x.detach()
    rows = {
        'wino4_conv op (fwd launch only)': host_us(lambda: ops.wino4_conv(xd, u4, None, 64, 6)),
        'WinogradConv2d fwd, no grad': host_us(lambda: conv(xd)),
        'nn.Conv2d (MIOpen) fwd, no grad': host_us(lambda: plain(xd)),
        'WinogradConv2d fwd+bwd': host_us(lambda: conv(x).sum().backward()),
        'nn.Conv2d fwd+bwd': host_us(lambda: plain(x).sum().backward()),
        'DropNormAct fwd+bwd': host_us(lambda: dna(x).sum().backward()),
        'conv_block (conv+DNA) fwd+bwd': host_us(lambda: cell(x).sum().backward()),
        'x.sum().backward() alone': host_us(lambda: x.sum().backward()),
    }
    for k, v in rows.items():
        print(f'{v:8.1f} us  {k}')
    print(json.dumps(rows))


if __name__ == '__main__':
    main()
