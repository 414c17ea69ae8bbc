"""U-Net 3x3 convolutions: HIP Winograd-on-MFMA kernel vs MIOpen (forward, backward-data).

    python benchmarks/conv_bench.py --out gpurun_out/conv_bench.json
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchgpipe_amd.ops import _ext  # noqa: E402

# (C, K, H) of U-Net(5,64) 3x3 convolutions (input 192x192), evaluated at micro-batch N.
LAYERS = [(3, 64, 192), (64, 64, 192), (64, 128, 96), (128, 128, 96), (128, 256, 48),
          (256, 256, 48), (256, 512, 24), (512, 512, 24), (512, 1024, 12), (1024, 1024, 12),
          (1024, 2048, 6), (2048, 2048, 6), (2048, 1024, 6), (2048, 512, 12), (1024, 256, 24),
          (512, 128, 48), (256, 64, 96), (128, 32, 192), (32, 32, 192)]


def timeit(fn, iters=10):  # type: ignore[no-untyped-def]
    for _ in range(2):
        fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--batch', type=int, nargs='+', default=[40, 16])
    p.add_argument('--out', default=None)
    p.add_argument('--sweep', action='store_true', help='time every tile variant x split count')
    args = p.parse_args()
    ops = _ext.require()
    dev = torch.device('cuda', 0)
    rows = []
    for n in args.batch:
        for c, k, h in LAYERS:
            x = torch.randn(n, c, h, h, device=dev)
            w = torch.randn(k, c, 3, 3, device=dev) / (3 * c ** 0.5)
            dy = torch.randn(n, k, h, h, device=dev)
            u = ops.wino_weight(w, False)
            ut = ops.wino_weight(w, True)
            flop = 2.0 * n * k * c * h * h * 9
            t_wf = timeit(lambda: ops.wino_conv(x, u, None, k))
            t_mf = timeit(lambda: F.conv2d(x, w, padding=1))
            t_wb = timeit(lambda: ops.wino_conv(dy, ut, None, c))
            t_mb = timeit(lambda: torch.ops.aten.convolution_backward(
                dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]))
            t_wt = timeit(lambda: ops.wino_weight(w, False))
            t_ww = timeit(lambda: ops.wino_wgrad(x, dy, 0))
            t_mw = timeit(lambda: torch.ops.aten.convolution_backward(
                dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
            sweep = {}
            if args.sweep:
                for var in (0, 1):
                    for sp in (1, 2, 4, 8):
                        sweep[f'v{var}s{sp}'] = round(timeit(
                            lambda: ops.wino_conv(x, u, None, k, var, sp)), 4)
            err = (ops.wino_conv(x, u, None, k) - F.conv2d(x, w, padding=1)).abs().max().item()
            row = {'N': n, 'C': c, 'K': k, 'H': h,
                   'wino_fwd_ms': round(t_wf, 4), 'miopen_fwd_ms': round(t_mf, 4),
                   'wino_bwd_data_ms': round(t_wb, 4), 'miopen_bwd_data_ms': round(t_mb, 4),
                   'weight_transform_ms': round(t_wt, 4),
                   'wino_wgrad_ms': round(t_ww, 4), 'miopen_wgrad_ms': round(t_mw, 4),
                   'wino_fwd_TFs': round(flop / t_wf / 1e9, 1),
                   'miopen_fwd_TFs': round(flop / t_mf / 1e9, 1),
                   'max_abs_err': err, 'sweep_fwd_ms': sweep}
            rows.append(row)
            print(json.dumps(row), flush=True)
            del x, w, dy, u, ut
    if args.out:
        with open(args.out, 'w') as f:
            json.dump({'device': torch.cuda.get_device_name(dev), 'rows': rows}, f, indent=1)


if __name__ == '__main__':
    main()
