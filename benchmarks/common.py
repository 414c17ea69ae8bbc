"""Shared harness of the reference-style benchmark CLIs.

Same metric definition as the reference benchmarks
(``benchmarks/unet-speed/main.py:201-254`` etc.): an epoch is ``dataset_size``
synthetic samples, bracketed by device synchronisation; throughput =
samples / elapsed; the first ``--skip-epochs`` epochs are discarded and the
rest averaged.  Two execution modes:

* ``--mode gpipe`` — the reference's single-process ``GPipe`` over
  ``--devices`` (one thread per GPU, peer copies over xGMI);
* ``--mode stage`` — one process per GPU under ``torch.distributed.run``
  (:class:`~torchgpipe_amd.parallel.PipelineStage`, RCCL point-to-point).
"""
import argparse
import json
import os
import platform
import sys
import time
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torchgpipe_amd  # noqa: E402
from torchgpipe_amd import GPipe  # noqa: E402

Experiment = Dict[str, object]
BASE_TIME = time.time()


def log(msg: str) -> None:
    t = time.time() - BASE_TIME
    print('%02d:%02d:%02d | %s' % (t // 3600, t % 3600 // 60, t % 60, msg), flush=True)


def parser(description: str, experiments: Dict[str, Experiment]) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=description)
    p.add_argument('experiment', choices=sorted(experiments))
    p.add_argument('--epochs', '-e', type=int, default=10)
    p.add_argument('--skip-epochs', '-k', type=int, default=1)
    p.add_argument('--devices', '-d', default=None, help='comma-separated GPU ids')
    p.add_argument('--mode', choices=['gpipe', 'stage'], default='gpipe')
    p.add_argument('--dataset-size', type=int, default=None)
    p.add_argument('--balance', default=None, help='override balance (comma-separated)')
    p.add_argument('--json', action='store_true', help='print a JSON summary line')
    return p


def parse_devices(value: Optional[str]) -> List[int]:
    if value is None:
        return list(range(torch.cuda.device_count()))
    return [int(x) for x in value.split(',')]


def run_speed(args: argparse.Namespace, experiment: Experiment,
              build: Callable[[], nn.Sequential], input_shape: Tuple[int, ...],
              make_target: Callable[[int, torch.device], torch.Tensor],
              loss_fn: Callable[[torch.Tensor, torch.Tensor], torch.Tensor],
              dataset_size: int) -> float:
    """Train for ``args.epochs`` epochs and return the mean samples/sec."""
    if args.skip_epochs >= args.epochs:
        raise SystemExit(f'--skip-epochs={args.skip_epochs} must be less than '
                         f'--epochs={args.epochs}')
    dataset_size = args.dataset_size or dataset_size
    batch = int(experiment['batch'])  # type: ignore[arg-type]
    balance = experiment.get('balance')
    if args.balance:
        balance = [int(v) for v in args.balance.split(',')]
    chunks = int(experiment.get('chunks', 1))  # type: ignore[arg-type]
    checkpoint = str(experiment.get('checkpoint', 'except_last'))
    model = build()

    if args.mode == 'stage':
        from torchgpipe_amd.parallel import PipelineStage
        world = int(os.environ.get('WORLD_SIZE', '1'))
        rank = int(os.environ.get('RANK', '0'))
        device = torch.device('cuda', int(os.environ.get('LOCAL_RANK', '0')))
        torch.cuda.set_device(device)
        if world > 1:
            dist.init_process_group('nccl')
        stage = PipelineStage(model, balance or [len(model)], device=device, chunks=chunks,
                              checkpoint=checkpoint)
        params = list(stage.parameters())
        in_device, out_device = device, device
        first, last = stage.is_first, stage.is_last
    else:
        devices = parse_devices(args.devices)
        if balance is None:  # baseline: plain model on one device
            in_device = out_device = torch.device('cuda', devices[0])
            model.to(in_device)
            stage = None
            params = list(model.parameters())
        else:
            model = GPipe(model, balance, devices=devices, chunks=chunks, checkpoint=checkpoint)
            in_device, out_device = model.devices[0], model.devices[-1]
            stage = None
            params = list(model.parameters())
        rank, world, first, last = 0, 1, True, True
        torch.cuda.set_device(in_device)

    optimizer = torch.optim.SGD(params, lr=0.1)
    x = torch.rand(batch, *input_shape, device=in_device)
    t = make_target(batch, out_device)
    steps = [(x, t)] * (dataset_size // batch)
    if dataset_size % batch:
        rem = dataset_size % batch
        steps.append((x[:rem], t[:rem]))

    if rank == 0:
        log(f'{args.experiment}: batch {batch}, chunks {chunks}, balance {balance}, '
            f'checkpoint {checkpoint}, mode {args.mode}')
        log(f'torchgpipe_amd {torchgpipe_amd.__version__}, python {platform.python_version()}, '
            f'torch {torch.__version__}, hip {torch.version.hip}, '
            f'gpu {torch.cuda.get_device_name(in_device)}')

    def sync() -> None:
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(in_device)

    throughputs = []
    for epoch in range(args.epochs):
        sync()
        tick = time.time()
        seen = 0
        for inp, tgt in steps:
            seen += inp.size(0)
            if stage is not None:
                stage.train_step(inp if first else None, tgt if last else None, loss_fn)
            else:
                loss = loss_fn(model(inp), tgt)
                loss.backward()
            optimizer.step()
            optimizer.zero_grad()
        sync()
        elapsed = time.time() - tick
        tp = seen / elapsed
        if rank == 0:
            log(f'{epoch + 1}/{args.epochs} epoch | {tp:.3f} samples/sec, {elapsed:.3f} sec/epoch')
        if epoch >= args.skip_epochs:
            throughputs.append(tp)
    mean = sum(throughputs) / len(throughputs)
    if rank == 0:
        log(f'{args.experiment}, {args.skip_epochs + 1}-{args.epochs} epochs | '
            f'{mean:.3f} samples/sec (average)')
        if args.json:
            print(json.dumps({'experiment': args.experiment, 'samples_per_sec': mean,
                              'batch': batch, 'chunks': chunks, 'balance': balance,
                              'mode': args.mode}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return mean
