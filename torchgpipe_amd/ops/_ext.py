"""Loader for the in-tree native extension ``torchgpipe_amd/_C.so``.

GPU tensors always go through the HIP kernels: if the extension is missing on
a machine with a GPU, every op raises instead of silently falling back to
PyTorch.  CPU tensors use the pure-PyTorch reference implementations (the
same math, used as the fp32 oracle in the numerics tests).
"""
import importlib
import os
from typing import Any, Optional

import torch

__all__ = ['available', 'ops', 'require', 'load_error']

_loaded = False
_error: Optional[BaseException] = None


def _load() -> None:
    global _loaded, _error
    if _loaded or _error is not None:
        return
    try:
        importlib.import_module('torchgpipe_amd._C')
        _loaded = True
    except Exception as exc:  # pragma: no cover - depends on the build
        _error = exc
        if os.environ.get('TGPIPE_AUTOBUILD', '0') == '1':
            from torchgpipe_amd._build import build
            build()
            _error = None
            importlib.import_module('torchgpipe_amd._C')
            _loaded = True


def available() -> bool:
    _load()
    return _loaded


def load_error() -> Optional[BaseException]:
    _load()
    return _error


def require(*tensors: torch.Tensor) -> Any:
    """Return ``torch.ops.tgpipe`` or raise if the HIP extension is unavailable."""
    _load()
    if not _loaded:
        raise RuntimeError(
            'torchgpipe_amd native extension (_C.so) is not built/loadable, '
            'but a GPU tensor needs it: run `python -m torchgpipe_amd._build` '
            f'(load error: {_error!r})')
    return torch.ops.tgpipe


def ops() -> Any:
    return require()
