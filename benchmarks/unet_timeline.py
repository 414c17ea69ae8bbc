"""U-Net(5,64) timeline ablation (reference: benchmarks/unet-timeline/main.py:21-170).

Measures the contribution of GPipe's three mechanisms on a 4-GPU single-process
pipeline (balance [34, 76, 70, 61], chunks 8, batch 128):

* ``baseline``   — no ``depend`` edges, copies on the compute streams, skips carried
                   as extra tuple elements through every partition (no portals)
* ``dep-x-x``    — + Fork/Join dependency edges
* ``dep-str-x``  — + dedicated copy streams
* ``dep-str-ptl``— + portals (skips copied directly stash GPU → pop GPU)

GPU utilisation is sampled with ``rocm-smi`` in a background thread.

    python benchmarks/unet_timeline.py dep-str-ptl --devices 0,1,2,3
"""
import argparse
import os
import subprocess
import sys
import threading
import time
from contextlib import contextmanager
from typing import Iterator, List

import torch
import torch.nn.functional as F
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torchgpipe_amd.pipeline as pipeline_mod  # noqa: E402
from torchgpipe_amd import GPipe  # noqa: E402
from torchgpipe_amd.models import unet  # noqa: E402
from torchgpipe_amd.models.unet import PopCat, Stash  # noqa: E402
from torchgpipe_amd.stream import current_stream  # noqa: E402

EXPERIMENTS = ['baseline', 'dep-x-x', 'dep-str-x', 'dep-str-ptl']


class _Carry(nn.Module):
    """Run ``layer`` on the head of a tuple and pass the carried skips through."""

    def __init__(self, layer: nn.Module) -> None:
        super().__init__()
        self.layer = layer

    def forward(self, xs):  # type: ignore[no-untyped-def]
        x, *skips = xs if isinstance(xs, tuple) else (xs,)
        y = self.layer(x)
        return (y, *skips) if skips else y


class _StashT(nn.Module):
    def forward(self, xs):  # type: ignore[no-untyped-def]
        x, *skips = xs if isinstance(xs, tuple) else (xs,)
        return (x, *skips, x)


class _PopCatT(nn.Module):
    def forward(self, xs):  # type: ignore[no-untyped-def]
        x, *skips = xs
        s = skips[-1]
        out = torch.cat((x, s), dim=1)
        rest = tuple(skips[:-1])
        return (out, *rest) if rest else out


def tuplify_skips(model: nn.Sequential) -> nn.Sequential:
    """Replace U-Net Stash/PopCat portals by skips carried along the tuple (LIFO)."""
    layers = []
    for name, layer in model.named_children():
        if isinstance(layer, Stash):
            layers.append((name, _StashT()))
        elif isinstance(layer, PopCat):
            layers.append((name, _PopCatT()))
        else:
            layers.append((name, _Carry(layer)))
    from collections import OrderedDict
    return nn.Sequential(OrderedDict(layers))


@contextmanager
def ablate(experiment: str) -> Iterator[None]:
    """Monkey-patch the runtime to remove mechanisms for the ablation."""
    orig_depend = pipeline_mod.depend
    if experiment == 'baseline':
        pipeline_mod.depend = lambda a, b: None  # type: ignore[assignment]
    try:
        yield
    finally:
        pipeline_mod.depend = orig_depend


class Utilization:
    """Mean GPU busy % over a period, sampled from rocm-smi."""

    def __init__(self, devices: List[int], period: float = 0.05) -> None:
        self.devices = devices
        self.period = period
        self.samples: List[float] = []
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, daemon=True)

    def _query(self) -> List[float]:
        try:
            out = subprocess.run(['rocm-smi', '--showuse', '--csv'], capture_output=True,
                                 text=True, timeout=5).stdout
        except Exception:
            return []
        values = []
        for line in out.splitlines()[1:]:
            parts = line.split(',')
            if len(parts) >= 2 and parts[0].startswith('card'):
                idx = int(''.join(ch for ch in parts[0] if ch.isdigit()) or 0)
                if idx in self.devices:
                    try:
                        values.append(float(parts[1]))
                    except ValueError:
                        pass
        return values

    def _run(self) -> None:
        while not self._stop.is_set():
            vals = self._query()
            if vals:
                self.samples.append(sum(vals) / len(vals))
            time.sleep(self.period)

    def __enter__(self) -> 'Utilization':
        self._thread.start()
        return self

    def __exit__(self, *exc: object) -> None:
        self._stop.set()
        self._thread.join()

    @property
    def mean(self) -> float:
        return sum(self.samples) / len(self.samples) if self.samples else float('nan')


def main() -> None:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    p.add_argument('experiment', choices=EXPERIMENTS)
    p.add_argument('--devices', '-d', default='0,1,2,3')
    p.add_argument('--epochs', type=int, default=3)
    p.add_argument('--steps', type=int, default=16, help='steps per epoch')
    args = p.parse_args()
    devices = [int(x) for x in args.devices.split(',')]
    balance, chunks, batch = [34, 76, 70, 61], 8, 128

    model = unet(depth=5, num_convs=5, base_channels=64)
    if args.experiment != 'dep-str-ptl':
        model = tuplify_skips(model)
    gpipe = GPipe(model, balance, devices=devices[:len(balance)], chunks=chunks)
    if args.experiment in ('baseline', 'dep-x-x'):
        # Copies on the compute streams instead of dedicated copy streams.
        gpipe._copy_streams = [[current_stream(d)] * chunks for d in gpipe.devices]
    opt = torch.optim.SGD(gpipe.parameters(), lr=0.1)
    x = torch.rand(batch, 3, 192, 192, device=gpipe.devices[0])
    t = torch.ones(batch, 1, 192, 192, device=gpipe.devices[-1])

    with ablate(args.experiment):
        for epoch in range(args.epochs):
            torch.cuda.synchronize(gpipe.devices[0])
            torch.cuda.reset_peak_memory_stats()
            with Utilization(devices) as util:
                tick = time.time()
                for _ in range(args.steps):
                    out = gpipe(x)
                    F.binary_cross_entropy_with_logits(out, t).backward()
                    opt.step()
                    opt.zero_grad()
                for d in gpipe.devices:
                    torch.cuda.synchronize(d)
                elapsed = time.time() - tick
            mem = sum(torch.cuda.max_memory_reserved(d) for d in gpipe.devices) / 2 ** 30
            print(f'{args.experiment} epoch {epoch + 1}: {batch * args.steps / elapsed:.3f} '
                  f'samples/sec, GPU util {util.mean:.0f}%, memory {mem:.1f} GiB', flush=True)


if __name__ == '__main__':
    main()
