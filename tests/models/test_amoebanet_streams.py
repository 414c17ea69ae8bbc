"""Two-stream schedule of the AmoebaNet cells (models/amoebanet.py, set_cell_streams)."""
import torch

from torchgpipe_amd.models import amoebanetd
from torchgpipe_amd.models.amoebanet import Cell, set_cell_streams


def test_stream_plans_split_the_cell_and_respect_dependencies():
    model = amoebanetd(num_classes=10, num_layers=3, num_filters=16)
    cells = [m for m in model.modules() if isinstance(m, Cell)]
    assert cells
    for cell in cells:
        for count in (2, 3, 4):
            plan = cell._stream_plan(count)
            # the two input reductions on different streams, one stream per node
            assert plan[:2] == [0, 1]
            assert len(plan) == 2 + len(cell.operations) // 2
            assert set(plan) <= set(range(count)) and len(set(plan)) >= 2
        # normal cells: the two 1x7-7x1 chains after the grouped op (nodes 3 and 4) run on
        # different streams once there are three
        if cell._group[1]:
            plan = cell._stream_plan(3)
            assert plan[3] != plan[4]


def test_set_cell_streams_toggles_every_cell_and_cpu_runs_one_stream():
    torch.manual_seed(0)
    model = amoebanetd(num_classes=10, num_layers=3, num_filters=16)
    x = torch.rand(2, 3, 224, 224)
    ref = model(x)
    set_cell_streams(model, True)
    assert all(m.streams == 3 for m in model.modules() if isinstance(m, Cell))
    set_cell_streams(model, 2)
    assert all(m.streams == 2 for m in model.modules() if isinstance(m, Cell))
    assert torch.equal(model(x), ref)  # CPU tensors: the one-stream path
    set_cell_streams(model, False)
    assert not any(m.streams for m in model.modules() if isinstance(m, Cell))


def test_shared_pools_compute_the_unshared_function():
    """A cell's duplicate 3x3 average pools of one node run once (Cell._shared_plan): same
    outputs and gradients as computing both (CPU)."""
    import copy
    import torch
    from torchgpipe_amd.models import amoebanetd
    from torchgpipe_amd.models.amoebanet import Cell
    torch.manual_seed(0)
    a = amoebanetd(num_classes=10, num_layers=3, num_filters=16)
    b = copy.deepcopy(a)
    plans = [m._shared for m in a.modules() if isinstance(m, Cell)]
    assert all(len(p) == 2 for p in plans)
    for m in b.modules():
        if isinstance(m, Cell):
            m._shared = []
    x = torch.randn(2, 3, 224, 224)
    ya, yb = a(x), b(x)
    torch.testing.assert_close(ya, yb, rtol=0, atol=0)
    ya.square().sum().backward()
    yb.square().sum().backward()
    for (name, pa), pb in zip(a.named_parameters(), b.parameters()):
        # (the shared pool's two gradients are summed before its backward instead of after:
        # fp32 reassociation only)
        rel = ((pa.grad - pb.grad).norm() / pb.grad.norm()).item()
        assert rel < 1e-5, (name, rel)
