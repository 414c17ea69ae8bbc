"""Run a function on N gloo ranks (CPU) and collect per-rank results."""
import os
import socket
import traceback

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, out_dir):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.set_num_threads(1)
    try:
        dist.init_process_group('gloo', rank=rank, world_size=world)
        result = fn(rank, world, *args)
        torch.save(result, os.path.join(out_dir, f'rank{rank}.pt'))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        with open(os.path.join(out_dir, f'rank{rank}.err'), 'w') as f:
            f.write(traceback.format_exc())
        raise


def run(fn, world, tmp_path, *args):
    out_dir = str(tmp_path)
    os.makedirs(out_dir, exist_ok=True)
    mp.start_processes(_entry, args=(world, free_port(), fn, args, out_dir), nprocs=world,
                       join=True, start_method='spawn')
    return [torch.load(os.path.join(out_dir, f'rank{r}.pt'), weights_only=False)
            for r in range(world)]
