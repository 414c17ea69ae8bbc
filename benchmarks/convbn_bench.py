"""Per-shape timing of AmoebaNet-D's convolutions: tgpipe implicit-GEMM MFMA kernels vs MIOpen.

Captures every ``nn.Conv2d`` input shape of AmoebaNet-D(18, 256) at one micro-batch
size (eager forward with hooks), then times forward / backward-data / weight-gradient
of each distinct shape with both implementations, weighted by how often the shape
occurs in the model.  Writes a JSON table (``--out``).

    python benchmarks/convbn_bench.py --micro-batch 20 --out profiles/convbn_bench.json
"""
import argparse
import json
import os
import sys
from collections import OrderedDict

import torch
from torch import nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def capture(micro_batch: int):
    from torchgpipe_amd.models import amoebanetd
    from torchgpipe_amd.ops import convbn
    model = amoebanetd(num_classes=1000, num_layers=18, num_filters=256).cuda()
    shapes: 'OrderedDict[tuple, int]' = OrderedDict()

    def hook(mod, inp):
        x = inp[0]
        if not convbn.conv_supported(mod):
            return
        key = (tuple(x.shape), tuple(mod.weight.shape), tuple(mod.stride), tuple(mod.padding))
        shapes[key] = shapes.get(key, 0) + 1

    handles = [m.register_forward_pre_hook(hook) for m in model.modules()
               if isinstance(m, nn.Conv2d)]
    with torch.no_grad(), convbn.disabled():
        model(torch.rand(micro_batch, 3, 224, 224, device='cuda'))
    for h in handles:
        h.remove()
    return shapes


def timeit(fn, reps: int = 20) -> float:
    for _ in range(3):
        fn()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    start.record()
    for _ in range(reps):
        fn()
    end.record()
    torch.cuda.synchronize()
    return start.elapsed_time(end) * 1000.0 / reps  # us


def main() -> None:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument('--micro-batch', type=int, default=20)
    p.add_argument('--out', default='')
    args = p.parse_args()
    from torchgpipe_amd.ops import _ext
    ops = _ext.require()
    rows = []
    tot = {'ours': 0.0, 'miopen': 0.0}
    for (xs, ws, stride, pad), count in capture(args.micro_batch).items():
        x = torch.randn(xs, device='cuda')
        w = torch.randn(ws, device='cuda') * 0.05
        kh, kw = ws[2], ws[3]
        geo = [kh, kw, stride[0], stride[1], pad[0], pad[1], 0, 0]
        y = ops.conv_gemm_forward(x, w, geo, False)
        dz = torch.randn_like(y)
        # backward-data's A operand W^T: training transposes each weight once per step for
        # all its micro-batches (ops/conv.py _TransformCache), so it is not timed per call
        w_t = w.transpose(0, 1).contiguous()
        flops = 2.0 * y.numel() * ws[1] * kh * kw
        r = {'x': xs, 'w': ws, 'stride': stride, 'pad': pad, 'count': count,
             'gflop': round(flops / 1e9, 3)}
        for name, fn in [
            ('fwd', lambda: ops.conv_gemm_forward(x, w, geo, True)),
            ('bwd_data', lambda: ops.conv_gemm_backward_data(dz, x, w, geo, True, w_t)),
            ('wgrad', lambda: ops.conv_gemm_backward_weight(dz, x, w, geo, True)),
            ('miopen_fwd', lambda: F.conv2d(x, w, stride=stride, padding=pad)),
            ('miopen_bwd_data', lambda: torch.ops.aten.convolution_backward(
                dz, x, w, None, list(stride), list(pad), [1, 1], False, [0, 0], 1,
                [True, False, False])),
            ('miopen_wgrad', lambda: torch.ops.aten.convolution_backward(
                dz, x, w, None, list(stride), list(pad), [1, 1], False, [0, 0], 1,
                [False, True, False])),
        ]:
            us = timeit(fn)
            r[name + '_us'] = round(us, 2)
            r[name + '_tflops'] = round(flops / us / 1e6, 1)
        ours = r['fwd_us'] + r['bwd_data_us'] + r['wgrad_us']
        theirs = r['miopen_fwd_us'] + r['miopen_bwd_data_us'] + r['miopen_wgrad_us']
        tot['ours'] += count * ours
        tot['miopen'] += count * theirs
        rows.append(r)
        print(json.dumps(r), flush=True)
    print(json.dumps({'weighted_total_us_ours': round(tot['ours'], 1),
                      'weighted_total_us_miopen': round(tot['miopen'], 1)}), flush=True)
    if args.out:
        with open(args.out, 'w') as f:
            json.dump({'micro_batch': args.micro_batch, 'rows': rows, 'totals': tot}, f, indent=1)


if __name__ == '__main__':
    main()
