"""Namespaces that isolate skip names (``Skippable.isolate``).

Parity: ``torchgpipe/skip/namespace.py:10-43``.  A namespace is identified by
a random UUID4; it is hashable and totally ordered (the order is arbitrary
but stable, which is all ``SkipLayout`` needs for sorting routes).  ``None``
is registered as a virtual subclass so that it acts as the default
namespace: ``isinstance(None, Namespace)`` is ``True``.
"""
import abc
from functools import total_ordering
from typing import Any
import uuid

__all__ = ['Namespace']


@total_ordering
class Namespace(metaclass=abc.ABCMeta):
    __slots__ = ('id',)

    def __init__(self) -> None:
        self.id = uuid.uuid4()

    def __repr__(self) -> str:
        return f"<Namespace '{self.id}'>"

    def __hash__(self) -> int:
        return hash(self.id)

    def __eq__(self, other: Any) -> bool:
        return isinstance(other, Namespace) and self.id == other.id

    def __lt__(self, other: Any) -> bool:
        return isinstance(other, Namespace) and self.id < other.id


Namespace.register(type(None))
