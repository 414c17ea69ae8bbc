import copy

import pytest
import torch
from torch import nn

from torchgpipe_amd import GPipe
from torchgpipe_amd.skip import Namespace, pop, skippable, stash


@skippable(stash=['1to3'])
class Layer1(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc = nn.Linear(4, 4)

    def forward(self, x):
        yield stash('1to3', x)
        return self.fc(x)


class Layer2(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc = nn.Linear(4, 4)

    def forward(self, x):
        return torch.tanh(self.fc(x))


@skippable(pop=['1to3'])
class Layer3(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc = nn.Linear(4, 4)

    def forward(self, x):
        skip = yield pop('1to3')
        return self.fc(x) + skip


@pytest.mark.parametrize('balance', [[3], [1, 2], [2, 1], [1, 1, 1]])
@pytest.mark.parametrize('checkpoint', ['always', 'except_last', 'never'])
def test_1to3_matches_plain_sequential(balance, checkpoint):
    torch.manual_seed(0)
    plain = nn.Sequential(Layer1(), Layer2(), Layer3())
    piped = GPipe(copy.deepcopy(plain), balance, devices=['cpu'] * len(balance), chunks=3,
                  checkpoint=checkpoint)
    x = torch.rand(6, 4, requires_grad=True)
    x2 = x.detach().clone().requires_grad_()
    y = plain(x)
    y2 = piped(x2)
    torch.testing.assert_close(y, y2)
    y.norm().backward()
    y2.norm().backward()
    torch.testing.assert_close(x.grad, x2.grad)
    for p, q in zip(plain.parameters(), piped.parameters()):
        torch.testing.assert_close(p.grad, q.grad)


def test_none_skip():
    @skippable(stash=['none'])
    class Stash(nn.Module):
        def forward(self, x):
            yield stash('none', None)
            return x

    @skippable(pop=['none'])
    class Pop(nn.Module):
        def forward(self, x):
            none = yield pop('none')
            assert none is None
            return x

    model = GPipe(nn.Sequential(Stash(), Pop()), [1, 1], devices=['cpu', 'cpu'], chunks=5)
    x = torch.rand(10, requires_grad=True)
    y = model(x)

    def assert_grad_fn_is_not_portal(grad_fn, visited=None):
        visited = set() if visited is None else visited
        if grad_fn in visited or grad_fn is None:
            return
        assert 'Portal' not in type(grad_fn).__name__
        visited.add(grad_fn)
        for next_fn, _ in grad_fn.next_functions:
            assert_grad_fn_is_not_portal(next_fn, visited)

    assert_grad_fn_is_not_portal(y.grad_fn)
    y.sum().backward()
    assert torch.allclose(x.grad, torch.ones_like(x))


def test_namespaced_unet_like_skips_across_partitions():
    @skippable(stash=['skip'])
    class Stash(nn.Module):
        def forward(self, x):
            yield stash('skip', x)
            return x * 2

    @skippable(pop=['skip'])
    class PopAdd(nn.Module):
        def forward(self, x):
            s = yield pop('skip')
            return x + s

    ns = [Namespace(), Namespace()]
    layers = [Stash().isolate(ns[0]), nn.Linear(2, 2), Stash().isolate(ns[1]), nn.Linear(2, 2),
              PopAdd().isolate(ns[1]), nn.Linear(2, 2), PopAdd().isolate(ns[0])]
    torch.manual_seed(0)
    plain = nn.Sequential(*layers)
    piped = GPipe(copy.deepcopy(plain), [2, 2, 2, 1], devices=['cpu'] * 4, chunks=4)
    x = torch.rand(8, 2)
    torch.testing.assert_close(plain(x), piped(x))


@pytest.mark.gpu
@pytest.mark.parametrize('devices', [[0, 0, 0], [0, 1, 2]], ids=['1gpu', '3gpu'])
def test_1to3_across_gpus(devices):
    """Skips from partition 0 to partition 2 through portals; with one GPU the three
    partitions share it (separate streams), so the test runs on every GPU box."""
    if max(devices) >= torch.cuda.device_count():
        pytest.skip(f'needs {max(devices) + 1} GPUs')
    torch.manual_seed(0)
    plain = nn.Sequential(Layer1(), Layer2(), Layer3())
    piped = GPipe(copy.deepcopy(plain), [1, 1, 1], devices=devices, chunks=3)
    x = torch.rand(6, 4)
    torch.testing.assert_close(plain(x), piped(x.cuda(0)).cpu())


@pytest.mark.parametrize('balance', [[104, 137], [30, 66, 84, 61]])
def test_same_route_skips_travel_as_one_hop(balance):
    """K7: every skip a micro-batch carries from one partition to another is one
    PortalCopy (one packed peer copy between GPUs), not one per skip.  U-Net(5, 2) has
    U-Net(5, 64)'s 241 layers, so the reference pipeline-4 balance applies."""
    from torchgpipe_amd import GPipe
    from torchgpipe_amd.models import unet
    from torchgpipe_amd.skip import portal
    from torchgpipe_amd.skip.layout import layout_from_balance

    model = unet(depth=5, num_convs=5, base_channels=2, input_channels=3, output_channels=1)
    n = len(balance)
    layout = layout_from_balance(model, balance)
    routes = sum(len(list(layout.copy_policy(j))) for j in range(n))
    groups = sum(len(layout.copy_groups(j)) for j in range(n))
    # p2: all 4 skips on route 0 -> 1; p4: 4 skips on 3 routes
    assert (routes, groups) == {2: (4, 1), 4: (4, 3)}[n]
    chunks = 2
    gpipe = GPipe(model, balance, devices=['cpu'] * n, chunks=chunks)
    before = portal.portal_hops
    out = gpipe(torch.rand(4, 3, 64, 64))
    assert portal.portal_hops - before == groups * chunks
    out.mean().backward()
    assert all(p.grad is not None for p in gpipe.parameters())


@pytest.mark.gpu
@pytest.mark.parametrize('base_channels,hw', [(4, 64), (32, 128)])
def test_unet_p2_skips_packed_peer_copies_match_one_gpu(base_channels, hw):
    """K5-K7 across two GPUs: U-Net pipeline-2 at the reference balance [104, 137] (all
    four long skips cross from GPU 0 to GPU 1 on one route).  Every micro-batch's skips
    make one PortalCopy hop; skips under ``copy.SKIP_PACK_MAX_BYTES`` travel as one packed
    peer copy (base 4: all of them; base 32 at 128^2: the 4.2 MB top-level skip one by
    one, the three others packed), and gradients
    match the whole model on one GPU with the same micro-batching."""
    if torch.cuda.device_count() < 2:
        pytest.skip('needs 2 GPUs')
    import torch.nn.functional as F

    from torchgpipe_amd import copy as copymod
    from torchgpipe_amd.models import unet
    from torchgpipe_amd.skip import portal

    torch.manual_seed(0)
    model = unet(depth=5, num_convs=5, base_channels=base_channels)
    for m in model.modules():  # no dropout: deterministic comparison
        if isinstance(getattr(m, 'p', None), float):
            m.p = 0.0
    plain = copy.deepcopy(model).cuda(0)
    chunks = 2
    gpipe = GPipe(model, [104, 137], devices=[0, 1], chunks=chunks)
    x = torch.rand(4, 3, hw, hw, device='cuda:0')
    t = torch.rand(4, 1, hw, hw)
    hops, packed = portal.portal_hops, copymod.packed_hops
    out = gpipe(x)
    assert portal.portal_hops - hops == chunks  # one skip hop per micro-batch
    # bytes of level k's skip per micro-batch (2 images, base_channels * 2^k channels)
    sizes = [base_channels * 2 ** k * (hw >> k) ** 2 * 2 * 4 for k in range(5)]
    small = sum(s < copymod.SKIP_PACK_MAX_BYTES for s in sizes[:4])
    assert copymod.packed_hops - packed == (chunks if small >= 2 else 0)
    F.binary_cross_entropy_with_logits(out, t.to(out.device)).backward()

    total = 0.0
    for xc, tc in zip(x.chunk(chunks), t.cuda(0).chunk(chunks)):
        loss = F.binary_cross_entropy_with_logits(plain(xc), tc) * (tc.size(0) / 4)
        loss.backward()
        total += loss.item()
    for (name, pa), pb in zip(plain.named_parameters(), gpipe.parameters()):
        scale = pa.grad.abs().max().item() + 1e-12
        torch.testing.assert_close(pb.grad.to(pa.device), pa.grad, rtol=1e-4,
                                   atol=1e-5 * scale, msg=name)
