"""Time every distinct convolution of AmoebaNet-D(18,256) (fwd, bwd-data, wgrad).

Finds the shapes on which MIOpen's immediate-mode heuristics fall back to slow
solvers (e.g. the ``naive_conv_*`` reference kernels) so they can be given a
native kernel.

    python benchmarks/amoeba_conv_bench.py --micro-batch 40 --out gpurun_out/amoeba_convs.json
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchgpipe_amd.models import amoebanetd  # noqa: E402


def conv_shapes(mb: int):
    model = amoebanetd(1000, 18, 256)
    shapes = {}

    def hook(mod, inp, out):  # type: ignore[no-untyped-def]
        if isinstance(mod, torch.nn.Conv2d):
            key = (tuple(inp[0].shape[1:]), mod.out_channels, mod.kernel_size, mod.stride,
                   mod.padding)
            shapes[key] = shapes.get(key, 0) + 1

    for m in model.modules():
        m.register_forward_hook(hook)
    model = model.to('meta')
    model(torch.empty(mb, 3, 224, 224, device='meta'))
    return shapes


def time_ms(fn, iters: int) -> float:
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--micro-batch', type=int, default=40)
    p.add_argument('--iters', type=int, default=5)
    p.add_argument('--out', default=None)
    args = p.parse_args()
    dev = torch.device('cuda', 0)
    rows = []
    for (cin_hw, cout, k, stride, pad), count in sorted(conv_shapes(args.micro_batch).items(),
                                                         key=lambda kv: -kv[1]):
        x = torch.randn(args.micro_batch, *cin_hw, device=dev)
        w = torch.randn(cout, cin_hw[0], *k, device=dev) * 0.05
        y = F.conv2d(x, w, None, stride, pad)
        dy = torch.randn_like(y)
        fwd = time_ms(lambda: F.conv2d(x, w, None, stride, pad), args.iters)
        bwd_data = time_ms(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, list(stride), list(pad), [1, 1], False, [0, 0], 1,
            [True, False, False]), args.iters)
        wgrad = time_ms(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, list(stride), list(pad), [1, 1], False, [0, 0], 1,
            [False, True, False]), args.iters)
        flops = 2.0 * y.numel() * cin_hw[0] * k[0] * k[1]
        row = dict(input=list(cin_hw), cout=cout, kernel=list(k), stride=list(stride),
                   pad=list(pad), per_forward=count, fwd_ms=round(fwd, 4),
                   bwd_data_ms=round(bwd_data, 4), wgrad_ms=round(wgrad, 4),
                   fwd_tflops=round(flops / fwd / 1e9, 1),
                   weighted_ms=round(count * (fwd * 2 + bwd_data + wgrad), 3))
        rows.append(row)
        print(json.dumps(row), flush=True)
    rows.sort(key=lambda r: -r['weighted_ms'])
    total = sum(r['weighted_ms'] for r in rows)
    print(f'total weighted ms per micro-batch (fwd x2 + bwd): {total:.2f}', flush=True)
    if args.out:
        with open(args.out, 'w') as f:
            json.dump({'micro_batch': args.micro_batch, 'rows': rows, 'total_ms': total}, f,
                      indent=1)


if __name__ == '__main__':
    main()
