"""Zero-element "phony" tensors used purely as autograd-edge carriers.

Parity: ``torchgpipe/phony.py:15-43``.  A phony has no storage, so passing it
through autograd functions creates graph edges (ordering constraints) with no
memory traffic and no gradient accumulation cost.  One phony per
``(device, requires_grad)`` is cached; it is allocated on the device's
default stream so that the caching allocator never has to track it across
side streams.
"""
import threading
from typing import Dict, List, Tuple

import torch
from torch import Tensor

from torchgpipe_amd.stream import default_stream, use_stream

__all__: List[str] = []

_cache: Dict[Tuple[torch.device, bool], Tensor] = {}
_lock = threading.Lock()


def get_phony(device: torch.device, *, requires_grad: bool) -> Tensor:
    """Return the cached phony for ``device``.

    An autograd function that returns a phony must return ``phony.detach()``;
    otherwise autograd would attach a ``grad_fn`` to the shared cached object.
    """
    key = (device, requires_grad)
    phony = _cache.get(key)
    if phony is not None:
        return phony
    with _lock:
        phony = _cache.get(key)
        if phony is None:
            with use_stream(default_stream(device)):
                phony = torch.empty(0, device=device, requires_grad=requires_grad)
            _cache[key] = phony
    return phony
