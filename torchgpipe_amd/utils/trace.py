"""Lightweight tracing: roctx ranges per pipeline cell / transfer.

The reference has no tracer.  Here every pipeline cell and every
inter-stage transfer can be bracketed by a roctx range so that ``rocprofv3
--marker-trace`` (or ``torch.profiler``) timelines show which micro-batch and
partition each kernel and xGMI copy belongs to.

Enable with ``TGPIPE_TRACE=1`` or ``trace.enable()``.  Disabled ranges cost
one attribute lookup (a shared ``nullcontext``).
"""
from contextlib import contextmanager, nullcontext
import os
import time
from typing import Dict, Generator, List, Optional

import torch

__all__ = ['enable', 'disable', 'enabled', 'range', 'Timeline']

_NULL = nullcontext()
_enabled = os.environ.get('TGPIPE_TRACE', '0') not in ('', '0')


def enable() -> None:
    global _enabled
    _enabled = True


def disable() -> None:
    global _enabled
    _enabled = False


def enabled() -> bool:
    return _enabled


@contextmanager
def _marker(label: str) -> Generator[None, None, None]:
    pushed = False
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(label)  # roctxRangePush on ROCm builds
            pushed = True
        except Exception:  # pragma: no cover - tracer library missing
            pushed = False
    with torch.autograd.profiler.record_function(label):
        try:
            yield
        finally:
            if pushed:
                torch.cuda.nvtx.range_pop()


def range(label: str):  # type: ignore[no-untyped-def]  # noqa: A001 - mirrors nvtx.range
    if not _enabled:
        return _NULL
    return _marker(label)


class Timeline:
    """Host-side wall-clock event log (start/stop per label), for tests & debugging."""

    def __init__(self) -> None:
        self.events: List[Dict[str, object]] = []
        self._t0 = time.perf_counter()

    @contextmanager
    def span(self, label: str, **meta: object) -> Generator[None, None, None]:
        start = time.perf_counter() - self._t0
        try:
            yield
        finally:
            stop = time.perf_counter() - self._t0
            self.events.append({'label': label, 'start': start, 'stop': stop, **meta})

    def labels(self, prefix: Optional[str] = None) -> List[str]:
        return [str(e['label']) for e in self.events
                if prefix is None or str(e['label']).startswith(prefix)]
