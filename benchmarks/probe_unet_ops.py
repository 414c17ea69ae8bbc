"""Per-phase timing probe of one U-Net(5,64) micro-batch on one GPU (diagnostics)."""
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from torchgpipe_amd.models import unet  # noqa: E402


def main():
    bench = len(sys.argv) > 1 and sys.argv[1] == 'bench'
    torch.backends.cudnn.benchmark = bench
    dev = torch.device('cuda', 0)
    model = unet().to(dev)
    mb = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    x = torch.rand(mb, 3, 192, 192, device=dev)
    t = torch.ones(mb, 1, 192, 192, device=dev)
    for it in range(4):
        torch.cuda.synchronize()
        t0 = time.time()
        y = model(x)
        torch.cuda.synchronize()
        t1 = time.time()
        F.binary_cross_entropy_with_logits(y, t).backward()
        torch.cuda.synchronize()
        t2 = time.time()
        print(f'iter {it}: fwd {1e3*(t1-t0):.1f} ms  bwd {1e3*(t2-t1):.1f} ms  '
              f'-> {mb/(t2-t0):.1f} samples/s', flush=True)


if __name__ == '__main__':
    main()
