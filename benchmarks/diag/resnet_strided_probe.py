"""Device time of ResNet-101's strided convolutions on MIOpen (forward, backward-data,
backward-weight, micro-batch 110 = pipeline-1 B 220 / m 2), and of the 1x1 stride-2
downsample as subsample + pointwise implicit GEMM (ops.convbn.gemm_conv2d).

    python benchmarks/diag/resnet_strided_probe.py [--batch 110]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = [  # name, cin, cout, k, stride, pad, h
    ('stem 7x7', 3, 64, 7, 2, 3, 224),
    ('l2 conv2 3x3', 128, 128, 3, 2, 1, 56),
    ('l2 down 1x1', 256, 512, 1, 2, 0, 56),
    ('l3 conv2 3x3', 256, 256, 3, 2, 1, 28),
    ('l3 down 1x1', 512, 1024, 1, 2, 0, 28),
    ('l4 conv2 3x3', 512, 512, 3, 2, 1, 14),
    ('l4 down 1x1', 1024, 2048, 1, 2, 0, 14),
]


def timed(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return round(a.elapsed_time(b) * 1000 / iters, 1)


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--batch', type=int, default=110)
    args = p.parse_args()
    dev = torch.device('cuda')
    rows = []
    for name, cin, cout, k, s, pad, h in SHAPES:
        x = torch.randn(args.batch, cin, h, h, device=dev)
        w = torch.randn(cout, cin, k, k, device=dev) * 0.05
        y = F.conv2d(x, w, stride=s, padding=pad)
        dy = torch.randn_like(y)
        conv_bwd = torch.ops.aten.convolution_backward
        row = {'name': name, 'x': list(x.shape), 'w': list(w.shape),
               'fwd_us': timed(lambda: F.conv2d(x, w, stride=s, padding=pad)),
               'bwd_data_us': timed(lambda: conv_bwd(dy, x, w, None, [s, s], [pad, pad],
                                                     [1, 1], False, [0, 0], 1,
                                                     [True, False, False])),
               'bwd_weight_us': timed(lambda: conv_bwd(dy, x, w, None, [s, s], [pad, pad],
                                                       [1, 1], False, [0, 0], 1,
                                                       [False, True, False]))}
        # whole Conv-BN-ReLU forward + backward: MIOpen conv + native BN (ops/fusion.py's
        # strided path) vs the fused implicit-GEMM op (backward-data: timed library choice)
        from torchgpipe_amd.ops.convbn import fusable, relu_conv_bn
        from torchgpipe_amd.ops.fusion import bn_act
        conv = torch.nn.Conv2d(cin, cout, k, stride=s, padding=pad, bias=False).to(dev)
        bn = torch.nn.BatchNorm2d(cout).to(dev)
        xg = x.clone().requires_grad_(cin > 3)

        def miopen_bn():
            y = bn_act(F.conv2d(xg, conv.weight, stride=s, padding=pad), bn, True)
            y.backward(dy)

        def fused():
            y = relu_conv_bn(xg, [(conv, 0)], bn, relu=False, relu_out=True)
            y.backward(dy)

        row['miopen_bn_fwd_bwd_us'] = timed(miopen_bn)
        row['fusable'] = fusable(xg, [conv], bn)
        if row['fusable']:
            row['fused_fwd_bwd_us'] = timed(fused)
            # the native backward-data (stride phases: conv_gemm_phases), no library choice
            ops = torch.ops.tgpipe
            geo = [k, k, s, s, pad, pad, 0, 0]
            row['native_bwd_data_us'] = timed(
                lambda: ops.conv_gemm_backward_data(dy, x, w, geo, False))
            row['native_fwd_us'] = timed(lambda: ops.conv_gemm_forward(x, w, geo, False))
            ops.lib_dgrad_force(0)
            try:
                row['fused_native_fwd_bwd_us'] = timed(fused)
            finally:
                ops.lib_dgrad_force(-1)
        if k == 1:
            from torchgpipe_amd.ops.convbn import gemm_conv2d
            conv = torch.nn.Conv2d(cin, cout, 1, bias=False).to(dev)
            with torch.no_grad():
                conv.weight.copy_(w)
            row['subsample_us'] = timed(lambda: x[:, :, ::s, ::s].contiguous())
            xs = x[:, :, ::s, ::s].contiguous()
            row['gemm_fwd_us'] = timed(lambda: gemm_conv2d(xs, conv))
        rows.append(row)
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
