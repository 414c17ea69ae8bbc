"""Microbenchmarks of the framework's HIP kernels vs the PyTorch sequences they replace.

Reports device time (HIP events, median of N) and achieved HBM bandwidth
(algorithmic bytes: every input read once, every output written once).

    python benchmarks/kernel_bench.py --out gpurun_out/kernel_bench.json
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchgpipe_amd.ops import fused  # noqa: E402
from torchgpipe_amd.ops import dropout as dropout_ops  # noqa: E402


def timeit(fn, iters=20):  # type: ignore[no-untyped-def]
    for _ in range(3):
        fn()
    times = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        times.append(a.elapsed_time(b))
    return statistics.median(times)


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--out', default=None)
    args = p.parse_args()
    dev = torch.device('cuda', 0)
    rows = []

    # K3: U-Net cell epilogue at every resolution (micro-batch 40, U-Net(5,64) channels).
    for n, c, hw in [(40, 64, 192), (40, 128, 96), (40, 256, 48), (40, 512, 24),
                     (40, 1024, 12), (40, 2048, 6), (16, 64, 192), (16, 32, 192)]:
        x = torch.randn(n, c, hw, hw, device=dev, requires_grad=True)
        nbytes = x.numel() * 4
        dy = torch.randn_like(x)

        def fused_fwd():
            return fused._DropNormAct.apply(x, 0.1, 1e-5, 1e-2, 1234, 0, True)

        def torch_fwd():
            return F.leaky_relu(F.instance_norm(F.dropout2d(x, 0.1, True)), 1e-2)

        y = fused_fwd()
        yt = torch_fwd()
        t_ff = timeit(fused_fwd)
        t_tf = timeit(torch_fwd)
        t_fb = timeit(lambda: torch.autograd.grad(y, x, dy, retain_graph=True))
        t_tb = timeit(lambda: torch.autograd.grad(yt, x, dy, retain_graph=True))
        rows.append({'op': 'dropout2d+instancenorm+leakyrelu', 'shape': [n, c, hw, hw],
                     'fused_fwd_ms': round(t_ff, 4), 'torch_fwd_ms': round(t_tf, 4),
                     'fused_bwd_ms': round(t_fb, 4), 'torch_bwd_ms': round(t_tb, 4),
                     'fused_fwd_TBps': round(2 * nbytes / t_ff / 1e9, 2),
                     'fused_bwd_TBps': round(3 * nbytes / t_fb / 1e9, 2)})
        print(json.dumps(rows[-1]), flush=True)
        del x, dy, y, yt

    # Native DeferredBatchNorm train forward (statistics + fp64 tracking + normalise) vs the
    # reference's path: ATen per-channel sums (torchgpipe/batchnorm.py:51-53) + MIOpen
    # BatchNorm.  Bytes: 2 reads + 1 write.
    ops = torch.ops.tgpipe
    for n, c, hw in [(40, 256, 56), (40, 1024, 14), (64, 64, 112)]:
        x = torch.randn(n, c, hw, hw, device=dev)
        w = torch.ones(c, device=dev)
        b = torch.zeros(c, device=dev)
        acc = torch.zeros(3, c, device=dev, dtype=torch.float64)
        s = torch.zeros(c, device=dev)
        q = torch.zeros(c, device=dev)
        nbytes = 3 * x.numel() * 4

        def old_path():
            s.add_(x.sum((0, 2, 3)))
            q.add_((x ** 2).sum((0, 2, 3)))
            F.batch_norm(x, None, None, w, b, True, 0.0, 1e-5)

        t_k = timeit(lambda: ops.bn_train_forward(x, w, b, acc, 1e-5))
        t_t = timeit(old_path)
        rows.append({'op': 'dbn_bn_train_forward', 'shape': [n, c, hw, hw],
                     'hip_ms': round(t_k, 4), 'aten_sums_plus_miopen_ms': round(t_t, 4),
                     'hip_TBps': round(nbytes / t_k / 1e9, 2)})
        print(json.dumps(rows[-1]), flush=True)

    # K4: elementwise Philox dropout.
    x = torch.randn(64 * 1024 * 1024, device=dev)
    t_k = timeit(lambda: dropout_ops._Dropout.apply(x, 0.1, 7, 0))
    t_t = timeit(lambda: F.dropout(x, 0.1, True))
    rows.append({'op': 'dropout', 'numel': x.numel(), 'hip_ms': round(t_k, 4),
                 'torch_ms': round(t_t, 4), 'hip_TBps': round(2 * x.numel() * 4 / t_k / 1e9, 2)})
    print(json.dumps(rows[-1]), flush=True)

    if args.out:
        with open(args.out, 'w') as f:
            json.dump({'device': torch.cuda.get_device_name(dev), 'rows': rows}, f, indent=1)


if __name__ == '__main__':
    main()
