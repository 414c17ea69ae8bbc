"""Static skip-connection routes across partitions.

Parity: ``torchgpipe/skip/layout.py:11-83``.  A route maps ``(ns, name)`` to
``(stash_partition, pop_partition)``.  Routes are indexed by destination and
sorted by source so that, before partition ``k`` runs a micro-batch, the
scheduler copies every cross-partition skip destined for ``k`` directly from
its source partition — over the direct xGMI link between those two GPUs,
never hopping through intermediate stages.

The same layout drives the multi-process engine, where a route ``j → k``
becomes an RCCL point-to-point send from rank ``j`` to rank ``k``.
"""
from typing import Dict, Iterable, List, Tuple

from torch import nn

from torchgpipe_amd.skip.namespace import Namespace

__all__: List[str] = []

Route = Tuple[int, Namespace, str]


class SkipLayout:
    def __init__(self, num_partitions: int,
                 skip_routes: Dict[Tuple[Namespace, str], Tuple[int, int]]) -> None:
        self.by_ns_name = skip_routes
        self.by_partition: List[List[Route]] = [[] for _ in range(num_partitions)]
        self.by_source: List[List[Tuple[int, Namespace, str]]] = [
            [] for _ in range(num_partitions)]
        for (ns, name), (src, dst) in skip_routes.items():
            self.by_partition[dst].append((src, ns, name))
            self.by_source[src].append((dst, ns, name))
        for routes in self.by_partition:
            routes.sort()
        for routes in self.by_source:
            routes.sort()

    def copy_policy(self, next_j: int) -> Iterable[Route]:
        """Cross-partition routes into ``next_j``, ascending by source partition."""
        for src, ns, name in self.by_partition[next_j]:
            if src != next_j:
                yield (src, ns, name)

    def copy_groups(self, next_j: int) -> List[Tuple[int, List[Tuple[Namespace, str]]]]:
        """:meth:`copy_policy` grouped by source partition: one transfer per route."""
        groups: List[Tuple[int, List[Tuple[Namespace, str]]]] = []
        for src, ns, name in self.copy_policy(next_j):
            if not groups or groups[-1][0] != src:
                groups.append((src, []))
            groups[-1][1].append((ns, name))
        return groups

    def send_policy(self, prev_j: int) -> Iterable[Tuple[int, Namespace, str]]:
        """Cross-partition routes out of ``prev_j``, ascending by destination."""
        for dst, ns, name in self.by_source[prev_j]:
            if dst != prev_j:
                yield (dst, ns, name)

    def requires_copy(self, ns: Namespace, name: str) -> bool:
        src, dst = self.by_ns_name.get((ns, name), (-1, -1))
        return src != dst

    def route(self, ns: Namespace, name: str) -> Tuple[int, int]:
        return self.by_ns_name.get((ns, name), (-1, -1))


def _skippable_layers(partition: nn.Sequential) -> Iterable[nn.Module]:
    from torchgpipe_amd.skip.skippable import Skippable  # cycle: skippable → tracker → layout
    for layer in partition:
        if isinstance(layer, Skippable):
            yield layer


def inspect_skip_layout(partitions: List[nn.Sequential]) -> SkipLayout:
    """Derive the static skip routes of ``partitions``."""
    routes: Dict[Tuple[Namespace, str], Tuple[int, int]] = {}
    stashed_at: Dict[Tuple[Namespace, str], int] = {}
    for j, partition in enumerate(partitions):
        for layer in _skippable_layers(partition):
            for key in layer.stashable():  # type: ignore[attr-defined]
                stashed_at[key] = j
            for key in layer.poppable():  # type: ignore[attr-defined]
                routes[key] = (stashed_at.pop(key), j)
    return SkipLayout(len(partitions), routes)


def layout_from_balance(module: nn.Sequential, balance: List[int]) -> SkipLayout:
    """Skip layout of ``module`` if it were split by ``balance`` (no split needed).

    Used by the multi-process engine, where each rank only materialises its own
    partition but must know every route that starts or ends at it.
    """
    layers = list(module.children())
    parts: List[nn.Sequential] = []
    start = 0
    for size in balance:
        parts.append(nn.Sequential(*layers[start:start + size]))
        start += size
    return inspect_skip_layout(parts)
