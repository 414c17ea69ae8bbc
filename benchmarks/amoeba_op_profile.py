"""Which PyTorch ops launch the non-fused kernels of an AmoebaNet-D training step.

torch.profiler over one GPipe step of AmoebaNet-D(18,256) at a reduced micro-batch count;
prints the aten ops by self device time with their call counts (copies, adds, cats).

    python benchmarks/amoeba_op_profile.py --chunks 4 --batch 80
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument('--chunks', type=int, default=4)
    p.add_argument('--batch', type=int, default=80)
    p.add_argument('--rows', type=int, default=30)
    a = p.parse_args()
    from torchgpipe_amd import GPipe
    from torchgpipe_amd.models import amoebanetd
    model = amoebanetd(num_classes=1000, num_layers=18, num_filters=256)
    g = GPipe(model, [len(model)], devices=[0], chunks=a.chunks, checkpoint='except_last')
    x = torch.rand(a.batch, 3, 224, 224, device='cuda')
    t = torch.randint(1000, (a.batch,), device='cuda')

    def step() -> None:
        F.cross_entropy(g(x), t).backward()
        g.zero_grad(set_to_none=True)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by='self_cuda_time_total', row_limit=a.rows,
                                    max_name_column_width=60))
    # who launches the copies / adds / cats (python stacks of those ops)
    for ev in prof.key_averages(group_by_stack_n=6):
        if ev.key in ('aten::copy_', 'aten::add_', 'aten::add', 'aten::cat', 'aten::fill_',
                      'aten::zero_') and ev.count >= 8:
            print(f'{ev.key} x{ev.count} self_cuda {ev.self_device_time_total / 1e3:.2f} ms')
            for frame in ev.stack[:6]:
                print('      ', frame)


if __name__ == '__main__':
    main()
