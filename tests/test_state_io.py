
import torch
from torch import nn

from tests.distributed.mp_util import run
from torchgpipe_amd import GPipe
from torchgpipe_amd.utils import state as state_io


def model():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(2, 4), nn.ReLU(), nn.Linear(4, 4), nn.BatchNorm1d(4),
                         nn.Linear(4, 1))


def test_gpipe_state_roundtrip_through_sequential_layout():
    g = GPipe(model(), [2, 3], devices=['cpu', 'cpu'])
    plain = state_io.to_sequential_state(g.state_dict())
    fresh = nn.Sequential(nn.Linear(2, 4), nn.ReLU(), nn.Linear(4, 4), nn.BatchNorm1d(4),
                          nn.Linear(4, 1))
    fresh.load_state_dict(plain)
    x = torch.rand(3, 2)
    g.eval()
    fresh.eval()
    torch.testing.assert_close(g(x), fresh(x))


def test_rebalance_state():
    g = GPipe(model(), [2, 3], devices=['cpu', 'cpu'])
    names = [n for n, _ in model().named_children()]
    sd = state_io.to_partitioned_state(state_io.to_sequential_state(g.state_dict()), names,
                                       [4, 1])
    g2 = GPipe(model(), [4, 1], devices=['cpu', 'cpu'])
    g2.load_state_dict(sd)
    assert 'partitions.1.4.weight' in sd and 'partitions.0.3.running_mean' in sd


def _save(rank, world, directory):
    from torchgpipe_amd.parallel import PipelineStage
    m = model()
    for p in m.parameters():
        p.data.add_(1.0)
    stage = PipelineStage(m, [2, 3], chunks=1)
    state_io.save_sharded(stage, directory)
    return None


def _load(rank, world, directory):
    from torchgpipe_amd.parallel import PipelineStage
    stage = PipelineStage(model(), [3, 2], chunks=1)  # different balance
    state_io.load_sharded(stage, directory)
    return {k: v.clone() for k, v in stage.partition.state_dict().items()}


def test_sharded_save_load_with_rebalance(tmp_path):
    d = str(tmp_path / 'ckpt')
    run(_save, 2, tmp_path / 'a', d)
    loaded = run(_load, 2, tmp_path / 'b', d)
    want = model()
    for p in want.parameters():
        p.data.add_(1.0)
    merged = {**loaded[0], **loaded[1]}
    for k, v in want.state_dict().items():
        torch.testing.assert_close(merged[k], v)


def _load_spy(rank, world, directory):
    import json
    from unittest import mock
    from torchgpipe_amd.parallel import PipelineStage
    stage = PipelineStage(model(), [4, 1], chunks=1)
    with open(f'{directory}/index.json') as f:
        layers = json.load(f)['layers']
    real_load = torch.load
    opened = []

    def spy(path, *args, **kwargs):
        opened.append(path.rsplit('/', 1)[1])
        return real_load(path, *args, **kwargs)

    with mock.patch.object(torch, 'load', spy):
        state_io.load_sharded(stage, directory)
    return {'opened': opened, 'layers': layers}


def test_load_sharded_reads_only_owning_shards(tmp_path):
    """with balance [4, 1] rank 1 owns layer 4, stored only in shard rank1.pt."""
    d = str(tmp_path / 'ckpt')
    run(_save, 2, tmp_path / 'a', d)
    got = run(_load_spy, 2, tmp_path / 'b', d)
    assert got[0]['layers'] == [['0', '1'], ['2', '3', '4']]
    assert got[0]['opened'] == ['rank0.pt', 'rank1.pt']
    assert got[1]['opened'] == ['rank1.pt']
