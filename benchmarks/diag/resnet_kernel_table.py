"""ResNet-101 pipeline-1 (B=220, m=2) training steps under torch.profiler: per-kernel device
time of the fused model (ops/fusion.py) or the plain nn model (--plain).  A rocprofv3
kernel trace of this benchmark loses its buffers: the process aborts at interpreter exit
in a library's static teardown (plain and fused alike)."""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchgpipe_amd import GPipe  # noqa: E402
from torchgpipe_amd.models.resnet import build_resnet  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument('--plain', action='store_true')
p.add_argument('--batch', type=int, default=220)
p.add_argument('--chunks', type=int, default=2)
p.add_argument('--rows', type=int, default=40)
args = p.parse_args()
model = build_resnet([3, 4, 23, 3], num_classes=1000, fused=not args.plain)
model = GPipe(model, [370], devices=[0], chunks=args.chunks)
opt = torch.optim.SGD(model.parameters(), lr=0.1)
x = torch.rand(args.batch, 3, 224, 224, device='cuda')
t = torch.randint(1000, (args.batch,), device='cuda')


def step():
    F.cross_entropy(model(x), t).backward()
    opt.step()
    opt.zero_grad()


for _ in range(4):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 5
print(f'{"plain" if args.plain else "fused"}: {1000 * dt:.1f} ms/step, '
      f'{args.batch / dt:.1f} samples/s', flush=True)
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    for _ in range(2):
        step()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by='cuda_time_total', row_limit=args.rows,
                                max_name_column_width=90), flush=True)
sys.stdout.flush()
