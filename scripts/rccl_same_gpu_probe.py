"""Probe: can two RCCL ranks share one GPU?  Launch with torch.distributed.run, 2 procs."""
import datetime
import os

import torch
import torch.distributed as dist

rank = int(os.environ['RANK'])
torch.cuda.set_device(0)
dist.init_process_group('nccl', timeout=datetime.timedelta(seconds=60))
x = torch.full((1024,), float(rank + 1), device='cuda:0')
if rank == 0:
    dist.send(x, 1)
else:
    dist.recv(x, 0)
torch.cuda.synchronize()
print(f'rank {rank}: got {x[0].item()} (expect 1.0)', flush=True)
dist.barrier()
dist.destroy_process_group()
