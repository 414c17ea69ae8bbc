"""User API for long skip connections: ``@skippable``, ``stash``, ``pop``.

Parity: ``torchgpipe/skip/skippable.py:27-416``.

A skippable module's ``forward`` is a *generator*: ``yield stash(name, t)``
hands a tensor to the skip connection, ``t = yield pop(name)`` receives it in
a later layer.  The decorator turns the user class into a
:class:`Skippable` subclass that drives the generator and routes the
commands through the current thread's skip tracker — a plain dict outside
``GPipe``, portals (single process) or RCCL point-to-point transfers
(``torchgpipe_amd.parallel``, multi process) inside it.  Names must be
declared statically so that the pipeline can derive the routes before
running (``verify_skippables``, ``inspect_skip_layout``).
"""
from typing import (Any, Callable, ClassVar, Dict, FrozenSet, Generator, Iterable, List,
                    Optional, Set, Tuple, Type, TypeVar, Union, cast)

from torch import Tensor, nn

from torchgpipe_amd.microbatch import Batch
from torchgpipe_amd.skip.namespace import Namespace
from torchgpipe_amd.skip.tracker import current_skip_tracker

__all__ = ['skippable', 'stash', 'pop', 'verify_skippables']

Tensors = Tuple[Tensor, ...]
TensorOrTensors = Union[Tensor, Tensors]
T = TypeVar('T', bound='Skippable')


class stash:
    """Command: ``yield stash(name, tensor)`` stores ``tensor`` under ``name``."""

    __slots__ = ('name', 'tensor')

    def __init__(self, name: str, tensor: Optional[Tensor]) -> None:
        self.name = name
        self.tensor = tensor


class pop:
    """Command: ``tensor = yield pop(name)`` retrieves the tensor stashed as ``name``."""

    __slots__ = ('name',)

    def __init__(self, name: str) -> None:
        self.name = name


class Skippable(nn.Module):
    """Base class of ``@skippable`` modules (create subclasses via the decorator)."""

    module_cls: ClassVar[Type[nn.Module]]
    stashable_names: ClassVar[FrozenSet[str]]
    poppable_names: ClassVar[FrozenSet[str]]

    def __init__(self, *args: Any, **kwargs: Any) -> None:
        super().__init__()
        self.module = self.module_cls(*args, **kwargs)
        self.namespaces: Dict[str, Namespace] = {}

    def __repr__(self) -> str:
        return f'@skippable({self.module})'

    def namespaced(self, name: str) -> Tuple[Namespace, str]:
        return (cast(Namespace, self.namespaces.get(name)), name)

    def stashable(self) -> Iterable[Tuple[Namespace, str]]:
        return [self.namespaced(n) for n in sorted(self.stashable_names)]

    def poppable(self) -> Iterable[Tuple[Namespace, str]]:
        return [self.namespaced(n) for n in sorted(self.poppable_names)]

    def isolate(self: T, ns: Namespace, *, only: Optional[Iterable[str]] = None) -> T:
        """Put all (or ``only`` the given) skip names of this module into ``ns``.

        Two pairs of layers that use the same skip name must live in different
        namespaces::

            ns1, ns2 = Namespace(), Namespace()
            nn.Sequential(Stash().isolate(ns1), Stash().isolate(ns2),
                          Pop().isolate(ns2), Pop().isolate(ns1))
        """
        names = (self.stashable_names | self.poppable_names) if only is None else set(only)
        for name in names:
            self.namespaces[name] = ns
        return self

    def dispatch(self, input: TensorOrTensors,
                 handle_stash: Callable[[str, Optional[Tensor]], None],
                 handle_pop: Callable[[str], Optional[Tensor]]) -> TensorOrTensors:
        """Drive the wrapped module's generator, servicing its commands."""
        result = self.module(input)
        if not isinstance(result, Generator):
            return result
        try:
            command = next(result)
            while True:
                if isinstance(command, stash):
                    handle_stash(command.name, command.tensor)
                    command = next(result)
                elif isinstance(command, pop):
                    command = result.send(handle_pop(command.name))
                else:
                    raise TypeError('%r is not a command from @skippable' % command)
        except StopIteration as stop:
            return stop.args[0] if stop.args else None  # type: ignore[return-value]

    def forward(self, input: TensorOrTensors) -> TensorOrTensors:  # type: ignore[override]
        tracker = current_skip_tracker()
        batch = Batch(input)

        to_pop: Dict[str, Optional[Tensor]] = {}
        for ns, name in self.poppable():
            try:
                to_pop[name] = tracker.load(batch, ns, name)
            except KeyError:
                raise RuntimeError(f"'{name}' has not been stashed")
        input = batch.tensor_or_tensors

        stashed: Dict[str, Optional[Tensor]] = {}

        def handle_stash(name: str, tensor: Optional[Tensor]) -> None:
            if name not in self.stashable_names:
                raise RuntimeError(f"'{name}' has not been declared as stashable")
            stashed[name] = tensor

        def handle_pop(name: str) -> Optional[Tensor]:
            if name not in self.poppable_names:
                raise RuntimeError(f"'{name}' has not been declared as poppable")
            return to_pop.pop(name)

        output = self.dispatch(input, handle_stash, handle_pop)

        missing = self.stashable_names - stashed.keys()
        if missing:
            names = ', '.join("'%s'" % n for n in missing)
            raise RuntimeError(f'{names} must be stashed but have not')
        if to_pop:
            names = ', '.join("'%s'" % n for n in to_pop)
            raise RuntimeError(f'{names} must be popped but have not')

        batch = Batch(output)
        for ns, name in self.stashable():
            tracker.save(batch, ns, name, stashed[name])
        return batch.tensor_or_tensors


def skippable(stash: Iterable[str] = (),
              pop: Iterable[str] = ()) -> Callable[[Type[nn.Module]], Type[Skippable]]:
    """Class decorator declaring the skip names a module stashes and pops.

    ::

        @skippable(stash=['1to3'])
        class Layer1(nn.Module):
            def forward(self, x):
                yield stash('1to3', x)
                return f1(x)

        @skippable(pop=['1to3'])
        class Layer3(nn.Module):
            def forward(self, x):
                skip = yield pop('1to3')
                return f3(x) + skip
    """
    stashable_names = frozenset(stash)
    poppable_names = frozenset(pop)

    def wrap(module_cls: Type[nn.Module]) -> Type[Skippable]:
        attrs = {'module_cls': module_cls,
                 'stashable_names': stashable_names,
                 'poppable_names': poppable_names}
        return type(module_cls.__name__, (Skippable,), attrs)

    return wrap


def verify_skippables(module: nn.Sequential) -> None:
    """Check statically that every skip name has exactly one stash and one pop.

    Raises ``TypeError`` listing every violation.
    """
    stashed: Set[Tuple[Namespace, str]] = set()
    popped: Set[Tuple[Namespace, str]] = set()
    problems: List[str] = []

    for layer_name, layer in module.named_children():
        if not isinstance(layer, Skippable):
            continue

        for name in sorted(layer.stashable_names & layer.poppable_names):
            problems.append(f"'{layer_name}' declared '{name}' both as stashable and as poppable")

        for ns, name in layer.stashable():
            if name in layer.poppable_names:
                continue
            if (ns, name) in stashed:
                problems.append(f"'{layer_name}' redeclared '{name}' as stashable "
                                'but not isolated by namespace')
                continue
            stashed.add((ns, name))

        for ns, name in layer.poppable():
            if name in layer.stashable_names:
                continue
            if (ns, name) in popped:
                problems.append(f"'{layer_name}' redeclared '{name}' as poppable "
                                'but not isolated by namespace')
                continue
            if (ns, name) not in stashed:
                problems.append(f"'{layer_name}' declared '{name}' as poppable "
                                'but it was not stashed')
                continue
            popped.add((ns, name))

    for _, name in sorted(stashed - popped, key=lambda k: k[1]):
        problems.append(f"no module declared '{name}' as poppable but stashed")

    if problems:
        raise TypeError('one or more pairs of stash and pop do not match:\n\n%s'
                        % '\n'.join('* %s' % p for p in problems))
