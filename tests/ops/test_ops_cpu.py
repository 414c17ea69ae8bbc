"""CPU references of the HIP ops (the GPU kernels are checked against these)."""
import torch
import torch.nn.functional as F

from torchgpipe_amd.ops import fused, misc, philox
from torchgpipe_amd.ops.dropout import dropout
from torchgpipe_amd.utils.rng import RngTape


def _philox_python(idx, off, seed):
    M = 0xFFFFFFFF
    c = [idx & M, (idx >> 32) & M, off & M, (off >> 32) & M]
    k = [seed & M, ((seed >> 32) & M) ^ 0x7467706D]
    for _ in range(10):
        p0 = 0xD2511F53 * c[0]
        p1 = 0xCD9E8D57 * c[2]
        c = [(p1 >> 32) ^ c[1] ^ k[0], p1 & M, (p0 >> 32) ^ c[3] ^ k[1], p0 & M]
        k = [(k[0] + 0x9E3779B9) & M, (k[1] + 0xBB67AE85) & M]
    return c


def test_philox_tensor_reference_matches_scalar_definition():
    idx = [0, 1, 7, 2 ** 32 + 5, 2 ** 40 + 7]
    words = philox.philox4x32_10(torch.tensor(idx), 123456789012, 2 ** 63 + 5)
    for i, v in enumerate(idx):
        assert [int(w[i]) for w in words] == _philox_python(v, 123456789012, 2 ** 63 + 5)


def test_philox_uniform_range_and_moments():
    u = philox.uniform(100_000, seed=3, offset=0)
    assert u.min() >= 0 and u.max() < 1
    assert abs(u.mean().item() - 0.5) < 0.01
    assert abs(u.var().item() - 1 / 12) < 0.005


def test_drop_norm_act_composite_matches_torch_modules_without_dropout():
    x = torch.randn(2, 3, 8, 8)
    want = F.leaky_relu(F.instance_norm(x), 0.01)
    got = fused.drop_norm_act(x, p=0.1, training=False)
    torch.testing.assert_close(got, want)


def test_drop_norm_act_drops_whole_channels():
    x = torch.randn(8, 16, 4, 4)
    y = fused.drop_norm_act(x, p=0.5, training=True)
    per_plane = y.abs().sum(dim=(2, 3))
    assert (per_plane == 0).any() and (per_plane > 0).any()


def test_drop_norm_act_replay():
    x = torch.randn(4, 4, 4, 4)
    tape = RngTape()
    with tape.recording():
        a = fused.drop_norm_act(x, 0.5)
    with tape.replaying():
        b = fused.drop_norm_act(x, 0.5)
    assert torch.equal(a, b)


def test_dropout_reference():
    torch.manual_seed(0)
    x = torch.ones(10_000)
    y = dropout(x, 0.3)
    kept = (y != 0).float().mean().item()
    assert abs(kept - 0.7) < 0.02
    torch.testing.assert_close(y[y != 0], torch.full_like(y[y != 0], 1 / 0.7))
    assert dropout(x, 0.3, training=False) is x


def test_pack_unpack_cpu():
    ts = [torch.randn(3, 5), torch.arange(7), torch.randn(2, 2).double()]
    buf = torch.empty(misc.packed_nbytes(ts), dtype=torch.uint8)
    misc.pack(ts, buf)
    outs = [torch.empty_like(t) for t in ts]
    misc.unpack(buf, outs)
    for a, b in zip(ts, outs):
        assert torch.equal(a, b)


def test_refresh_step_caches_names_the_stage_sources(monkeypatch):
    """The pre-split refresh (csrc/convbn.cpp conv_gemm_presplit_refresh) gets exactly this
    module's device parameters plus its cached derived weights -- another stage's entries
    stay untouched (a whole-step graph must capture the derives of its own stage)."""
    from types import SimpleNamespace

    from torch import nn

    from torchgpipe_amd.ops import _ext, conv, convbn

    class FakeCuda:  # a parameter stand-in that reports is_cuda
        def __init__(self, t):
            self.t, self.is_cuda = t, True

    seen = []
    monkeypatch.setattr(_ext, '_loaded', True)
    monkeypatch.setattr(torch, 'ops', SimpleNamespace(tgpipe=SimpleNamespace(
        conv_gemm_presplit_refresh=lambda sources: seen.append(list(sources)) or len(sources))))
    m = nn.Sequential(nn.Conv2d(4, 8, 1, bias=False), nn.Conv2d(8, 8, 1, bias=False))
    derived = torch.zeros(3)
    cache = convbn._weight_cache(m[0])
    cache._entries[(True, True, 'T')] = ((0, 0, torch.device('cpu'), 0), derived, None)
    monkeypatch.setattr(conv._TransformCache, 'refresh', lambda self: None)
    fakes = [FakeCuda(p) for p in m.parameters()]
    monkeypatch.setattr(nn.Module, 'parameters', lambda self, recurse=True: iter(fakes))
    conv.refresh_step_caches(m)
    assert len(seen) == 1
    assert seen[0][0] is derived
    assert seen[0][1:] == fakes

