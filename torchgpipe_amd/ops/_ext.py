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

__all__ = ['available', 'ops', 'require', 'load_error', 'load_plans', 'save_plans',
           'load_lib_dgrad', 'save_lib_dgrad']

# Implicit-GEMM launch plans measured on an MI355X for the benchmark models (written by
# benchmarks/tune_plans.py).  TGPIPE_CG_DB=<file> loads another table, =0 none.  Training
# never times candidates itself (csrc/convbn.cpp tuned_plan): a shape missing from the
# table runs the heuristic plan unless TGPIPE_CG_TUNE=1.
_TUNED = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tuned')
SHIPPED_PLANS = os.path.join(_TUNED, 'conv_gemm_mi355x.txt')
# Geometries whose backward-data measured faster on MIOpen (same tuner): "n ci h w co kh kw
# sh sw ph pw" per line.  TGPIPE_LIB_DGRAD_DB=<file> / =0 as above.
SHIPPED_LIB_DGRAD = os.path.join(_TUNED, 'lib_dgrad_mi355x.txt')

_loaded = False
_error: Optional[BaseException] = None


def _load() -> None:
    global _loaded, _error
    if _loaded or _error is not None:
        return
    try:
        importlib.import_module('torchgpipe_amd._C')
        _loaded = True
        db = os.environ.get('TGPIPE_CG_DB', SHIPPED_PLANS)
        if db != '0' and os.path.exists(db):
            load_plans(db)
        db = os.environ.get('TGPIPE_LIB_DGRAD_DB', SHIPPED_LIB_DGRAD)
        if db != '0' and os.path.exists(db):
            load_lib_dgrad(db)
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


def load_plans(path: str) -> int:
    """Seed the convolution autotuner with a saved plan table; returns plans taken.

    Entries that are not valid launch shapes of this build are ignored, and shapes already
    measured in this process keep their plan.
    """
    with open(path) as f:
        return int(torch.ops.tgpipe.conv_gemm_plans_import(f.read()))


def save_plans(path: str) -> int:
    """Write every plan measured (or loaded) in this process; returns the line count."""
    text = require().conv_gemm_plans_export()
    with open(path, 'w') as f:
        f.write(text)
    return text.count('\n')


def load_lib_dgrad(path: str) -> int:
    """Seed the backward-data library choice with a saved table; returns lines taken."""
    with open(path) as f:
        return int(torch.ops.tgpipe.lib_dgrad_import(f.read()))


def save_lib_dgrad(path: str) -> int:
    """Write the geometries whose backward-data runs on the library; returns the count."""
    text = require().lib_dgrad_export()
    with open(path, 'w') as f:
        f.write(text)
    return text.count('\n')
