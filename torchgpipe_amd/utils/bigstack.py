"""Run a call on a worker thread with a large native stack.

Why: replaying a large *multi-stream* hipGraph crashed with SIGSEGV inside
``hipGraphLaunch`` -- the full AmoebaNet-D(18,256) step with two-stream cells,
~100 k kernel nodes joined by cross-stream event edges
(``profiles/r2/bench_amoeba_n1m32_s13_streams_graph_crash.log``).  A faulthandler
stack put the fault in ``torch.cuda.CUDAGraph.replay`` with no Python frame below
it, the tiny model of the same code replayed fine, and the same full-size run
with ``ulimit -s unlimited`` completed and ran at 343.5 samples/s
(``profiles/r3/capture_crash.md``): the runtime walks the graph's DAG
recursively when it launches it, and a deep fork/join DAG overflows the default
8 MiB main-thread stack.  A single-stream capture is a plain chain and does not
recurse that deep, which is why the one-stream workaround of round 2 hid it.

The fix here does not depend on the caller's ``ulimit``: graph launches run on one
persistent worker thread whose stack is reserved at 1 GiB of address space (pages are
committed only when touched).  ``StepGraph`` runs its warm-up steps and the capture on
that thread as well: ending the capture of a three-stream AmoebaNet step overflowed the
main thread's stack the same way (``hipStreamEndCapture`` / instantiation), and a library
call (hipBLASLt for a Linear layer) made for the first time on a thread *inside* a
capture has to create its per-thread handle there, which crashes -- the warm-up steps
create those handles on the worker first.  The caller's device and current stream are
propagated, exceptions are re-raised in the caller, and the call is synchronous from the
caller's point of view (the worker only *enqueues* GPU work, like the caller would have).
"""
import contextlib
import queue
import threading
from typing import Any, Callable, Optional, Tuple

import torch

__all__ = ['call_with_big_stack', 'STACK_BYTES']

STACK_BYTES = 1 << 30

_lock = threading.Lock()
_worker: Optional['_Worker'] = None


class _Worker:
    def __init__(self) -> None:
        self.requests: 'queue.Queue[Tuple[Callable[[], Any], queue.Queue]]' = queue.Queue()
        prev = threading.stack_size()
        threading.stack_size(STACK_BYTES)
        try:
            self.thread = threading.Thread(target=self._run, name='tgpipe-big-stack',
                                           daemon=True)
            self.thread.start()
        finally:
            threading.stack_size(prev)

    def _run(self) -> None:
        while True:
            fn, reply = self.requests.get()
            try:
                reply.put((True, fn()))
            except BaseException as exc:  # re-raised in the caller
                reply.put((False, exc))


def call_with_big_stack(fn: Callable[[], Any]) -> Any:
    """``fn()`` on the big-stack worker, under the caller's CUDA device and stream.

    The caller's thread-local autograd state follows the call: grad mode, inference mode
    and autocast (enabled flag and dtype per device type), so a step captured or replayed
    under ``torch.autocast`` or ``torch.no_grad`` runs exactly as it would have on the
    caller's thread.  A call made from the worker itself runs in place (queueing it would
    deadlock the worker on its own request).
    """
    global _worker
    with _lock:
        if _worker is None:
            _worker = _Worker()
        worker = _worker
    if threading.current_thread() is worker.thread:
        return fn()
    device = torch.cuda.current_device() if torch.cuda.is_available() else None
    stream = torch.cuda.current_stream() if device is not None else None
    grad = torch.is_grad_enabled()
    inference = torch.is_inference_mode_enabled()
    autocast = [(kind, torch.is_autocast_enabled(kind), torch.get_autocast_dtype(kind))
                for kind in ('cuda', 'cpu')]

    def wrapped() -> Any:
        with contextlib.ExitStack() as stack:
            stack.enter_context(torch.inference_mode(inference))
            stack.enter_context(torch.set_grad_enabled(grad))
            for kind, enabled, dtype in autocast:
                if enabled:
                    stack.enter_context(torch.autocast(kind, dtype=dtype))
            if device is not None:
                stack.enter_context(torch.cuda.device(device))
                stack.enter_context(torch.cuda.stream(stream))
            return fn()

    reply: 'queue.Queue' = queue.Queue(maxsize=1)
    worker.requests.put((wrapped, reply))
    ok, value = reply.get()
    if not ok:
        raise value
    return value
