"""Training-state (checkpoint) I/O for pipelines: balance-independent save / load.

The reference has no save/load code: ``GPipe`` is an ``nn.Module`` whose
state-dict keys are ``partitions.<j>.<child-name>.<param>``
(``tests/test_gpipe.py:423-434`` in the reference).  This module keeps that
format as the canonical on-disk layout and adds what pipelines need:

* :func:`to_sequential_state` / :func:`to_partitioned_state` convert between
  the GPipe layout and a plain ``nn.Sequential`` layout (strip / add the
  ``partitions.<j>.`` prefix), so a checkpoint can be re-balanced or loaded
  into an unwrapped model;
* :func:`stage_state_dict` gives a multi-process stage's shard under the same
  GPipe keys, and :func:`save_sharded` / :func:`load_sharded` write/read one
  file per rank plus an index, loading each shard straight onto the rank's
  device (``map_location``) — with a different balance than it was saved with
  if needed.
"""
from collections import OrderedDict
import json
import os
import re
from typing import Dict, List, Mapping, Optional, Sequence

import torch
from torch import Tensor, nn

__all__ = ['to_sequential_state', 'to_partitioned_state', 'stage_state_dict',
           'load_stage_state_dict', 'save_sharded', 'load_sharded']

_PREFIX = re.compile(r'^partitions\.(\d+)\.(.*)$')


def to_sequential_state(state: Mapping[str, Tensor]) -> 'OrderedDict[str, Tensor]':
    """``partitions.<j>.<name>.<p>`` → ``<name>.<p>`` (plain ``nn.Sequential`` keys)."""
    out: 'OrderedDict[str, Tensor]' = OrderedDict()
    for key, value in state.items():
        match = _PREFIX.match(key)
        if match is None:
            raise KeyError(f'not a GPipe state-dict key: {key!r}')
        out[match.group(2)] = value
    return out


def _layer_names(module: nn.Sequential) -> List[str]:
    return [name for name, _ in module.named_children()]


def to_partitioned_state(state: Mapping[str, Tensor], layer_names: Sequence[str],
                         balance: Sequence[int]) -> 'OrderedDict[str, Tensor]':
    """``<name>.<p>`` → ``partitions.<j>.<name>.<p>`` for the given balance."""
    owner: Dict[str, int] = {}
    idx = 0
    for j, size in enumerate(balance):
        for name in layer_names[idx:idx + size]:
            owner[name] = j
        idx += size
    out: 'OrderedDict[str, Tensor]' = OrderedDict()
    for key, value in state.items():
        layer = key.split('.', 1)[0]
        out[f'partitions.{owner[layer]}.{key}'] = value
    return out


def stage_state_dict(stage) -> 'OrderedDict[str, Tensor]':  # type: ignore[no-untyped-def]
    """State of a :class:`~torchgpipe_amd.parallel.PipelineStage` under GPipe keys."""
    return OrderedDict((f'partitions.{stage.rank}.{k}', v)
                       for k, v in stage.partition.state_dict().items())


def load_stage_state_dict(stage, state: Mapping[str, Tensor],  # type: ignore[no-untyped-def]
                          strict: bool = True) -> None:
    """Load this stage's layers from a GPipe- or Sequential-layout state-dict."""
    mine = set(_layer_names(stage.partition))
    plain = {}
    for key, value in state.items():
        match = _PREFIX.match(key)
        key = match.group(2) if match else key
        if key.split('.', 1)[0] in mine:
            plain[key] = value
    stage.partition.load_state_dict(plain, strict=strict)


def save_sharded(stage, directory: str, extra: Optional[dict] = None) -> str:  # type: ignore[no-untyped-def]
    """Write ``rank<j>.pt`` (this stage's tensors) and, on rank 0, ``index.json``."""
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, f'rank{stage.rank}.pt')
    torch.save({k: v.detach().cpu() for k, v in stage_state_dict(stage).items()}, path)
    if stage.rank == 0:
        index = {'format': 'torchgpipe_amd/partitioned-v1', 'balance': list(stage.balance),
                 'world': stage.n, 'extra': extra or {},
                 # which layers each shard holds: loaders read only the shards they need
                 'layers': getattr(stage, 'layer_names', None)}
        with open(os.path.join(directory, 'index.json'), 'w') as f:
            json.dump(index, f, indent=1)
    return path


def load_sharded(stage, directory: str, strict: bool = True) -> None:  # type: ignore[no-untyped-def]
    """Load this stage from a sharded checkpoint, even if saved with another balance.

    Only the shards that hold one of this stage's layers are read (the index records
    every shard's layer names), with ``weights_only=True`` onto the host; only this
    stage's tensors then move to its device, so no rank stages foreign shards through
    its GPU.  Indexes without layer names (older checkpoints) read every shard.
    """
    with open(os.path.join(directory, 'index.json')) as f:
        index = json.load(f)
    mine = set(_layer_names(stage.partition))
    layers = index.get('layers')
    ranks = (range(index['world']) if not layers
             else [r for r, names in enumerate(layers) if mine & set(names)])
    merged: Dict[str, Tensor] = {}
    for r in ranks:
        shard = torch.load(os.path.join(directory, f'rank{r}.pt'), map_location='cpu',
                           weights_only=True)
        for key, value in to_sequential_state(shard).items():
            if key.split('.', 1)[0] in mine:
                merged[key] = value.to(stage.device)
        del shard
    stage.partition.load_state_dict(merged, strict=strict)
