"""Per-rank stream and communicator counts of the bench's 8-rank pipelines fit the
hardware queues bench.py asks for (``GPU_MAX_HW_QUEUES``), multi-path transfers included.

A HIP stream beyond the process's hardware queues shares one with another stream, and the
queue then runs their work in order: an RCCL receive spinning on one stream would hold up
compute queued on the other.  The engine's side streams are named process-wide
(``stream.named_stream``), so a process that builds many stages keeps this set.  The
counts come from the real models' skip layouts at the reference balances (built on the
meta device) and, for striping, from the engine's own
planner with every eligible route above the threshold (the most relays it can plan).
"""
import pytest
import torch
from torch import nn

from torchgpipe_amd.gpipe import partition_layers
from torchgpipe_amd.parallel import stripes
from torchgpipe_amd.parallel.stage import (CENSUS_LIMIT, HW_QUEUES, link_pairs,
                                           stream_census)
from torchgpipe_amd.skip.layout import inspect_skip_layout


def _layout(kind, balance):
    from torchgpipe_amd.models import amoebanetd, unet
    with torch.device('meta'):
        model = (unet(depth=5, num_convs=5, base_channels=64) if kind == 'unet'
                 else amoebanetd(num_classes=1000, num_layers=18, num_filters=256))
    parts = [nn.Sequential(g) for g in partition_layers(model, balance)]
    return inspect_skip_layout(parts)


def _worst_plan(pairs_directed, n):
    big = 1 << 30
    sends = {j: [] for j in range(n)}
    for src, dst, kind in pairs_directed:
        sends[src].append(stripes.Send(dst, kind, big))
        sends[dst].append(stripes.Send(src, 'g' + kind, big))
    return stripes.plan(sends, list(range(n)), 1)


@pytest.mark.parametrize('kind,balance', [
    ('unet', [16, 27, 31, 44, 22, 57, 27, 17]),
    ('unet', [18, 26, 27, 30, 22, 44, 40, 34]),
    ('amoebanet', [2, 2, 2, 3, 3, 4, 4, 4]),
    ('amoebanet', [2, 2, 3, 3, 3, 3, 3, 5]),
])
@pytest.mark.parametrize('striped', [False, True])
def test_eight_rank_streams_fit_the_hardware_queues(kind, balance, striped):
    import bench
    assert bench.HW_QUEUES == HW_QUEUES
    n = len(balance)
    layout = _layout(kind, balance)
    pairs = link_pairs(layout, n)
    directed = [(j, j + 1, 'act') for j in range(n - 1)]
    directed += [(s, d, 'skip') for s, d in set(layout.by_ns_name.values()) if s != d]
    routes, jobs = _worst_plan(directed, n) if striped else ({}, {})
    unet = kind == 'unet'
    for rank in range(n):
        relay_pairs = {frozenset((end, r)) for (src, dst), relays in routes.items()
                       for r in relays for end in (src, dst)}
        census = stream_census(rank, pairs, forward_lanes=unet, recompute_lanes=unet,
                               cell_streams=0 if unet else 3, graph_cells=False,
                               relay_routes=len(jobs.get(rank, [])),
                               relay_links=sum(1 for k in relay_pairs if rank in k))
        assert census['total'] <= CENSUS_LIMIT < HW_QUEUES, (rank, census)
    if striped:
        assert routes  # the worst case did plan relays

