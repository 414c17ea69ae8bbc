"""Flatten nested ``nn.Sequential`` containers into one flat ``nn.Sequential``.

Child names are joined with ``_`` (``encoder_0_encode_0_conv``), which is the
naming the reference benchmark models use (``benchmarks/models/*/
flatten_sequential.py``), so balance tables and state-dict keys line up.
"""
from collections import OrderedDict
from typing import Iterator, Tuple

from torch import nn

__all__ = ['flatten_sequential']


def _walk(module: nn.Sequential, prefix: str = '') -> Iterator[Tuple[str, nn.Module]]:
    for name, child in module.named_children():
        full = f'{prefix}_{name}' if prefix else name
        if isinstance(child, nn.Sequential):
            yield from _walk(child, full)
        else:
            yield full, child


def flatten_sequential(module: nn.Sequential) -> nn.Sequential:
    if not isinstance(module, nn.Sequential):
        raise TypeError('not sequential')
    return nn.Sequential(OrderedDict(_walk(module)))
