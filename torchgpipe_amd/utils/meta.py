"""Build huge models without host memory: construct on ``meta``, materialise per partition.

A 15.8 B-parameter U-Net(48,160) needs 63 GB just for fp32 weights; building it
on the host before splitting (the reference's only path) needs that much RAM
per process.  Instead::

    with torch.device('meta'):
        model = unet(depth=48, base_channels=160)
    gpipe = GPipe(model, balance, devices=...)   # each partition materialised on its GPU

:func:`materialize` allocates a module's parameters/buffers directly on the
target device (``to_empty``) and re-runs every submodule's
``reset_parameters()`` there, so initialisation also happens on the GPU.
"""
import torch
from torch import nn

__all__ = ['is_meta', 'materialize']


def is_meta(module: nn.Module) -> bool:
    return any(t.is_meta for t in list(module.parameters()) + list(module.buffers()))


@torch.no_grad()
def materialize(module: nn.Module, device: torch.device) -> nn.Module:
    """Allocate ``module`` on ``device`` and (re)initialise it there."""
    module.to_empty(device=device)
    for sub in module.modules():
        reset = getattr(sub, 'reset_parameters', None)
        if callable(reset):
            reset()
        # BatchNorm running stats live in buffers reset by reset_running_stats.
        reset_stats = getattr(sub, 'reset_running_stats', None)
        if callable(reset_stats):
            reset_stats()
    return module
