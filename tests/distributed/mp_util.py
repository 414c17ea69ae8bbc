"""Run a function on N ranks (gloo on CPU, or RCCL with one GPU per rank) and collect results."""
import datetime
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


def _entry(rank, world, port, fn, args, out_dir, backend, timeout, barrier):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.set_num_threads(1)
    try:
        kwargs = {'timeout': datetime.timedelta(seconds=timeout)}
        if backend.startswith('nccl'):
            torch.cuda.set_device(rank)
            if backend == 'nccl':  # eager communicator; 'nccl-lazy' = bench.py's mode
                kwargs['device_id'] = torch.device('cuda', rank)
            backend = 'nccl'
        dist.init_process_group(backend, rank=rank, world_size=world, **kwargs)
        result = fn(rank, world, *args)
        torch.save(result, os.path.join(out_dir, f'rank{rank}.pt'))
        if not barrier:
            # The test broke the group on purpose (timeouts close gloo pairs).
            os._exit(0)
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        with open(os.path.join(out_dir, f'rank{rank}.err'), 'w') as f:
            f.write(traceback.format_exc())
        raise


def run(fn, world, tmp_path, *args, backend='gloo', timeout=120, barrier=True):
    """Run ``fn(rank, world, *args)`` on ``world`` spawned ranks; returns their results.

    ``backend='nccl'`` / ``'nccl-lazy'`` puts rank r on ``cuda:r`` (RCCL, eagerly or
    lazily initialised communicators); ``timeout`` bounds every
    collective / point-to-point wait, so a deadlock fails the test instead of hanging it.
    """
    out_dir = str(tmp_path)
    os.makedirs(out_dir, exist_ok=True)
    mp.start_processes(_entry,
                       args=(world, free_port(), fn, args, out_dir, backend, timeout, barrier),
                       nprocs=world, join=True, start_method='spawn')
    return [torch.load(os.path.join(out_dir, f'rank{r}.pt'), weights_only=False)
            for r in range(world)]
