"""Distributed accuracy benchmark: CIFAR-10 classification over ``DistributedGPipe``.

Counterpart of the reference's ``benchmarks/distributed/accuracy/main.py:28-381`` (ResNet-101
/ ResNet-50 / VGG-16, one pipeline stage per process, SGD momentum 0.9 / nesterov / weight
decay 1e-4 with the gradual-warm-up linear LR scaling, per-epoch train throughput and
validation loss / accuracy).  Differences: stages talk over RCCL (GPU direct) instead of
CPU-staged RPC, the launcher is ``torchrun`` (one rank per GPU) instead of RPC workers, and
the data is either the CIFAR-10 binary release (``--data DIR`` holding
``data_batch_{1..5}.bin`` / ``test_batch.bin``: raw bytes, parsed with numpy; no
torchvision here) resized to 224x224 on the GPU, or ``synthetic``: a learnable stand-in
(per-class template + noise) for machines without the dataset (no network here), so
accuracy is "parity unpinned" against the reference.

    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 benchmarks/distributed_accuracy.py \\
        naive-128 --model resnet101 --balance 90,100,100,80 --chunks 4 --data synthetic
"""
import argparse
import os
import sys
import time
from typing import Dict, Iterator, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import Tensor, nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchgpipe_amd.distributed import DistributedGPipe  # noqa: E402
from torchgpipe_amd.models import resnet50, resnet101, vgg16  # noqa: E402

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def mlp_tiny(num_classes: int, inplace: bool = False) -> nn.Sequential:
    """Plumbing model for CPU runs (the test suite)."""
    return nn.Sequential(nn.Flatten(), nn.Linear(3 * 16 * 16, 64), nn.ReLU(inplace=inplace),
                         nn.Linear(64, 64), nn.ReLU(inplace=inplace), nn.Linear(64, num_classes))


MODELS = {
    'resnet101': lambda n, inplace: resnet101(num_classes=n, inplace=inplace),
    'resnet50': lambda n, inplace: resnet50(num_classes=n, inplace=inplace),
    'vgg16': lambda n, inplace: vgg16(num_classes=n, inplace=inplace),
    'mlp-tiny': mlp_tiny,
}
EXPERIMENTS = {'naive-128': dict(batch=128)}


def load_cifar10_bin(directory: str, train: bool) -> Tuple[np.ndarray, np.ndarray]:
    """CIFAR-10 binary release: records of 1 label byte + 3x32x32 pixel bytes."""
    names = [f'data_batch_{i}.bin' for i in range(1, 6)] if train else ['test_batch.bin']
    raw = np.concatenate([np.fromfile(os.path.join(directory, n), dtype=np.uint8)
                          for n in names]).reshape(-1, 1 + 3 * 32 * 32)
    return raw[:, 1:].reshape(-1, 3, 32, 32), raw[:, 0].astype(np.int64)


def synthetic(n: int, size: int, seed: int) -> Tuple[np.ndarray, np.ndarray]:
    """Ten fixed random templates plus per-sample noise: learnable, unlike pure noise."""
    rng = np.random.default_rng(1234)
    templates = rng.integers(0, 256, size=(10, 3, size, size)).astype(np.float32)
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, 10, size=n)
    noise = rng.normal(0.0, 60.0, size=(n, 3, size, size)).astype(np.float32)
    images = np.clip(templates[labels] * 0.15 + 100.0 + noise, 0, 255).astype(np.uint8)
    return images, labels.astype(np.int64)


class Batches:
    """Shuffled mini-batches of (uint8 images, labels), preprocessed on ``device``."""

    def __init__(self, images: np.ndarray, labels: np.ndarray, batch: int, size: int,
                 device: torch.device, shuffle: bool, seed: int) -> None:
        self.images, self.labels = images, labels
        self.batch, self.size, self.device = batch, size, device
        self.shuffle, self.seed, self.epoch = shuffle, seed, 0
        self.mean = torch.tensor(MEAN, device=device).view(1, 3, 1, 1)
        self.std = torch.tensor(STD, device=device).view(1, 3, 1, 1)

    def __len__(self) -> int:
        return len(self.labels) // self.batch  # full batches only (even micro-batches)

    def __iter__(self) -> Iterator[Tuple[Tensor, Tensor]]:
        order = np.arange(len(self.labels))
        if self.shuffle:  # identical order on every rank (same seed + epoch)
            np.random.default_rng(self.seed + self.epoch).shuffle(order)
        self.epoch += 1
        for i in range(len(self)):
            idx = order[i * self.batch:(i + 1) * self.batch]
            x = torch.from_numpy(self.images[idx]).to(self.device).float().div_(255.0)
            if x.shape[-1] != self.size:
                x = F.interpolate(x, size=(self.size, self.size), mode='bilinear',
                                  align_corners=False)
            yield (x - self.mean) / self.std, torch.from_numpy(self.labels[idx]).to(self.device)


def lr_multiplier(step: int, steps_per_epoch: int, batch: int) -> float:
    """Gradual warm-up to linear scaling over 4 epochs, /10 at epochs 30, 60, 80."""
    epoch = step / max(1, steps_per_epoch)
    scale = max(1.0, batch / 256)
    mult = min(4.0, epoch) / 4.0 * (scale - 1.0) + 1.0
    for boundary, factor in ((80, 0.001), (60, 0.01), (30, 0.1)):
        if epoch >= boundary:
            return factor * mult
    return mult


def train(args: argparse.Namespace) -> Dict[str, float]:
    """One pipeline stage per rank of the initialised process group (or one process)."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    if args.device == 'cuda':
        device = torch.device('cuda', int(os.environ.get('LOCAL_RANK', rank)))
        torch.cuda.set_device(device)
    else:
        device = torch.device('cpu')
    last = rank == world - 1
    batch = args.batch_size or EXPERIMENTS[args.experiment]['batch']
    if batch % args.chunks:
        raise SystemExit('--batch-size must be a multiple of --chunks')
    torch.manual_seed(0)
    model = MODELS[args.model](10, False)
    balance = ([int(v) for v in args.balance.split(',')] if args.balance
               else [len(model) // world + (1 if r < len(model) % world else 0)
                     for r in range(world)])
    pipe = DistributedGPipe(model, rank, {r: f'worker{r}' for r in range(world)}, balance,
                            args.chunks, device=device, checkpoint=args.checkpoint)

    if args.data == 'synthetic':
        tr_x, tr_y = synthetic(args.synthetic_size, 32, seed=1)
        va_x, va_y = synthetic(max(batch, args.synthetic_size // 4), 32, seed=2)
    else:
        tr_x, tr_y = load_cifar10_bin(args.data, train=True)
        va_x, va_y = load_cifar10_bin(args.data, train=False)
    size = args.image_size
    train_data = Batches(tr_x, tr_y, batch, size, device, True, seed=0)
    valid_data = Batches(va_x, va_y, batch, size, device, False, seed=0)
    steps = len(train_data) if args.max_steps <= 0 else min(len(train_data), args.max_steps)

    optimizer = torch.optim.SGD(pipe.parameters(), lr=args.lr, momentum=0.9,
                                weight_decay=1e-4, nesterov=True)
    scheduler = torch.optim.lr_scheduler.LambdaLR(
        optimizer, lambda s: lr_multiplier(s, steps, batch))

    def log(msg: str) -> None:
        if last:
            print(msg, flush=True)

    def run_epoch(epoch: int) -> Tuple[float, float, float]:
        pipe.train()
        t0 = time.time()
        loss_sum, seen = 0.0, 0
        for it, (x, y) in zip(range(steps), train_data):
            outputs = pipe.forward(x if rank == 0 else None)
            losses: Optional[List[Tensor]] = None
            if last:
                losses = [F.cross_entropy(o, t) for o, t in zip(outputs, y.chunk(args.chunks))]
                loss_sum += float(sum(l_.detach() for l_ in losses)) / args.chunks * batch
            pipe.backward(losses)
            optimizer.step()
            optimizer.zero_grad(set_to_none=True)
            scheduler.step()
            seen += batch
        if device.type == 'cuda':
            torch.cuda.synchronize(device)
        elapsed = time.time() - t0
        return loss_sum / max(1, seen), seen / elapsed, elapsed

    def evaluate() -> Tuple[float, float]:
        pipe.eval()
        loss_sum, correct, seen = 0.0, 0, 0
        with torch.no_grad():
            for x, y in valid_data:
                outputs = pipe.forward(x if rank == 0 else None)
                if last:
                    logits = torch.cat([o.float() for o in outputs])
                    loss_sum += float(F.cross_entropy(logits, y, reduction='sum'))
                    correct += int((logits.argmax(1) == y).sum())
                seen += len(y)
        return loss_sum / max(1, seen), correct / max(1, seen)

    log(f'{args.experiment} | {args.model} | {world} stage(s), balance {balance}, '
        f'{args.chunks} micro-batches, batch {batch}, {args.epochs} epochs, '
        f'data {args.data}, device {device}')
    throughputs: List[float] = []
    accuracy = 0.0
    for epoch in range(args.epochs):
        train_loss, throughput, elapsed = run_epoch(epoch)
        valid_loss, accuracy = evaluate()
        log(f'{epoch + 1}/{args.epochs} epoch | lr {scheduler.get_last_lr()[0]:.5f} | '
            f'train loss {train_loss:.3f} {throughput:.1f} samples/sec | '
            f'valid loss {valid_loss:.3f} accuracy {accuracy:.4f}')
        if epoch >= args.skip_epochs:
            throughputs.append(throughput)
    mean = sum(throughputs) / len(throughputs) if throughputs else 0.0
    log(f'{args.experiment} | valid accuracy: {accuracy:.4f} | {mean:.3f} samples/sec '
        f'(average of epochs {args.skip_epochs + 1}-{args.epochs})')
    return {'accuracy': accuracy, 'samples_per_sec': mean}


def parse(argv: Optional[List[str]] = None) -> argparse.Namespace:
    p = argparse.ArgumentParser(description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument('experiment', choices=sorted(EXPERIMENTS))
    p.add_argument('--model', '-m', choices=sorted(MODELS), default='resnet101')
    p.add_argument('--balance', '-b', default='', help='comma-separated layers per stage')
    p.add_argument('--chunks', '-c', type=int, default=4)
    p.add_argument('--batch-size', '-s', type=int, default=0)
    p.add_argument('--epochs', '-e', type=int, default=10)
    p.add_argument('--skip-epochs', '-k', type=int, default=1)
    p.add_argument('--lr', type=float, default=0.1)
    p.add_argument('--data', default='synthetic', help="CIFAR-10 binary directory or 'synthetic'")
    p.add_argument('--synthetic-size', type=int, default=5120)
    p.add_argument('--image-size', type=int, default=224)
    p.add_argument('--max-steps', type=int, default=0, help='cap the steps per epoch')
    p.add_argument('--checkpoint', choices=['always', 'except_last', 'never'],
                   default='except_last')
    p.add_argument('--device', choices=['cuda', 'cpu'],
                   default='cuda' if torch.cuda.device_count() else 'cpu')
    a = p.parse_args(argv)
    if a.skip_epochs >= a.epochs:
        p.error(f'--skip-epochs={a.skip_epochs} must be less than --epochs={a.epochs}')
    return a


def main() -> None:
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world > 1:
        backend = 'nccl' if args.device == 'cuda' else 'gloo'
        if args.device == 'cuda':
            torch.cuda.set_device(int(os.environ.get('LOCAL_RANK', '0')))
        dist.init_process_group(backend)
    train(args)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
