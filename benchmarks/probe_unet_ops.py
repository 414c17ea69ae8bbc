"""Per-phase timing probe of one U-Net(5,64) micro-batch on one GPU (diagnostics).

    python benchmarks/probe_unet_ops.py --mb 40 --variants fused unfused fused_cl unfused_cl
"""
import argparse
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from torchgpipe_amd.models import unet  # noqa: E402


def run(variant: str, mb: int, iters: int) -> None:
    dev = torch.device('cuda', 0)
    fused = variant.startswith('fused')
    cl = variant.endswith('_cl')
    model = unet(fused=fused).to(dev)
    fmt = torch.channels_last if cl else torch.contiguous_format
    model = model.to(memory_format=fmt)
    x = torch.rand(mb, 3, 192, 192, device=dev).contiguous(memory_format=fmt)
    t = torch.ones(mb, 1, 192, 192, device=dev)
    best = None
    for it in range(iters):
        torch.cuda.synchronize()
        t0 = time.time()
        y = model(x)
        torch.cuda.synchronize()
        t1 = time.time()
        F.binary_cross_entropy_with_logits(y, t).backward()
        torch.cuda.synchronize()
        t2 = time.time()
        model.zero_grad(set_to_none=True)
        if it >= 1:
            cur = (1e3 * (t1 - t0), 1e3 * (t2 - t1))
            best = cur if best is None or sum(cur) < sum(best) else best
        print(f'{variant} iter {it}: fwd {1e3*(t1-t0):.1f} ms bwd {1e3*(t2-t1):.1f} ms',
              file=sys.stderr, flush=True)
    print(f'{variant} mb={mb}: fwd {best[0]:.1f} ms  bwd {best[1]:.1f} ms  -> '
          f'{mb / (sum(best) / 1e3):.1f} samples/s', flush=True)


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--mb', type=int, default=40)
    p.add_argument('--iters', type=int, default=4)
    p.add_argument('--variants', nargs='+', default=['fused', 'unfused'])
    args = p.parse_args()
    for v in args.variants:
        run(v, args.mb, args.iters)


if __name__ == '__main__':
    main()
