"""Build huge models without host memory: construct on ``meta``, materialise per partition.

A 15.8 B-parameter U-Net(48,160) needs 63 GB just for fp32 weights; building it
on the host before splitting (the reference's only path) needs that much RAM
per process.  Instead::

    with torch.device('meta'):
        model = unet(depth=48, base_channels=160)
    gpipe = GPipe(model, balance, devices=...)   # each partition materialised on its GPU

:func:`materialize` allocates the meta parameters/buffers directly on the
target device (``to_empty``) and re-runs the owning submodules'
``reset_parameters()`` there, so initialisation also happens on the GPU.
"""
import torch
from torch import nn

__all__ = ['is_meta', 'materialize']


def is_meta(module: nn.Module) -> bool:
    return any(t.is_meta for t in list(module.parameters()) + list(module.buffers()))


@torch.no_grad()
def materialize(module: nn.Module, device: torch.device) -> nn.Module:
    """Allocate the meta tensors of ``module`` on ``device`` and initialise them there.

    Only submodules that directly own a meta parameter or buffer are touched:
    already-materialised (e.g. loaded) weights of a partly-meta partition keep
    their values.  Such a submodule is re-initialised with its own
    ``reset_parameters()`` and ``reset_running_stats()`` (BatchNorm, including
    DeferredBatchNorm's accumulators); meta buffers of a module without either
    are zero-filled, and a meta parameter without ``reset_parameters`` is an
    error (it would otherwise hold allocator garbage).
    """
    for sub in module.modules():
        own = list(sub.parameters(recurse=False)) + list(sub.buffers(recurse=False))
        if not any(t.is_meta for t in own):
            continue
        sub.to_empty(device=device, recurse=False)
        reset = getattr(sub, 'reset_parameters', None)
        reset_stats = getattr(sub, 'reset_running_stats', None)
        if callable(reset):
            reset()
        elif callable(reset_stats):
            reset_stats()
        else:
            for name, p in sub.named_parameters(recurse=False):
                raise RuntimeError(f'cannot initialise meta parameter {name!r} of '
                                   f'{type(sub).__name__}: it has no reset_parameters()')
            for b in sub.buffers(recurse=False):
                b.zero_()
        if callable(reset) and callable(reset_stats):
            reset_stats()
    return module.to(device)
