
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
