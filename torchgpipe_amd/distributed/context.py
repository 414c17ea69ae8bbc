"""Named per-process mailboxes (API parity with ``torchgpipe/distributed/context.py``).

The reference routes activations, gradients and targets between stage
processes through RPC calls that deposit tensors into these mailboxes
(``put_forward`` … ``get_target``).  The MI355X engine moves tensors with RCCL
point-to-point instead (:mod:`torchgpipe_amd.parallel.p2p`), so the
mailboxes are no longer on the data path; they are kept, with identical
semantics, for code that uses them directly (custom schedules, host-side
hand-offs, tests).

Each :class:`TrainingContext` owns ``chunks`` forward and backward channels
and one target channel; :class:`GlobalContext` maps context names to them.
"""
from contextlib import contextmanager
from queue import Queue
from typing import Any, Callable, Dict, Generator, Tuple, Union

from torch import Tensor

__all__ = ['TrainingContext', 'GlobalContext', 'worker', 'distributed', 'put_forward',
           'get_forward', 'put_backward', 'get_backward', 'put_target', 'get_target']

Tensors = Tuple[Tensor, ...]
TensorOrTensors = Union[Tensor, Tensors]


class TrainingContext:
    def __init__(self, context_name: str, microbatch_chunks: int) -> None:
        self.name = context_name
        self.forward_channels = [Queue() for _ in range(microbatch_chunks)]  # type: ignore[var-annotated]
        self.backward_channels = [Queue() for _ in range(microbatch_chunks)]  # type: ignore[var-annotated]
        self.target_channel: Queue = Queue()


class GlobalContext:
    ctxs: Dict[str, TrainingContext] = {}

    @staticmethod
    def get_context(context_name: str) -> TrainingContext:
        """Raises ``KeyError`` for an unknown context."""
        return GlobalContext.ctxs[context_name]


@contextmanager
def worker(context_name: str, microbatch_chunks: int) -> Generator[None, None, None]:
    """Register a training context for the duration of the block (names are unique)."""
    if context_name in GlobalContext.ctxs:
        raise RuntimeError(f'worker {context_name} already exists')
    GlobalContext.ctxs[context_name] = TrainingContext(context_name, microbatch_chunks)
    try:
        yield
    finally:
        del GlobalContext.ctxs[context_name]


def distributed(context_name: str, microbatch_chunks: int) -> Callable:
    """Decorator form of :func:`worker`."""
    def decorator(func: Callable) -> Callable:
        def wrapped(*args: Any, **kwargs: Any) -> Any:
            with worker(context_name, microbatch_chunks):
                return func(*args, **kwargs)
        return wrapped
    return decorator


def put_forward(context_name: str, id: int, value: TensorOrTensors) -> None:
    GlobalContext.get_context(context_name).forward_channels[id].put(value)


def get_forward(context_name: str, id: int) -> TensorOrTensors:
    return GlobalContext.get_context(context_name).forward_channels[id].get()


def put_backward(context_name: str, id: int, value: TensorOrTensors) -> None:
    GlobalContext.get_context(context_name).backward_channels[id].put(value)


def get_backward(context_name: str, id: int) -> TensorOrTensors:
    return GlobalContext.get_context(context_name).backward_channels[id].get()


def put_target(context_name: str, value: TensorOrTensors) -> None:
    GlobalContext.get_context(context_name).target_channel.put(value)


def get_target(context_name: str) -> TensorOrTensors:
    return GlobalContext.get_context(context_name).target_channel.get()
