import time

import pytest
import torch
from torch import nn

from torchgpipe_amd.balance import balance_by_size, balance_by_time, blockpartition
from torchgpipe_amd.balance.profile import layerwise_sandbox

gpu = pytest.mark.gpu


def test_blockpartition():
    assert blockpartition.solve([1, 2, 3, 4, 5, 6], partitions=2) == [[1, 2, 3, 4], [5, 6]]


def test_blockpartition_zeros():
    assert blockpartition.solve([0, 0], partitions=2) == [[0], [0]]


@pytest.mark.parametrize('partitions', [0, -1])
def test_blockpartition_non_positive_partitions(partitions):
    with pytest.raises(ValueError, match='partitions must be a positive integer'):
        blockpartition.solve([42], partitions=partitions)


def test_blockpartition_short_sequence():
    with pytest.raises(ValueError, match='sequence is shorter than intended partitions'):
        blockpartition.solve([], partitions=1)
    with pytest.raises(ValueError, match='sequence is shorter than intended partitions'):
        blockpartition.solve([42], partitions=2)


def _brute_force_minmax(seq, k):
    import itertools
    n = len(seq)
    best = None
    for cuts in itertools.combinations(range(1, n), k - 1):
        bounds = (0,) + cuts + (n,)
        cost = max(sum(seq[a:b]) for a, b in zip(bounds, bounds[1:]))
        best = cost if best is None else min(best, cost)
    return best


@pytest.mark.parametrize('seed', range(10))
def test_blockpartition_is_optimal(seed):
    import random
    rnd = random.Random(seed)
    seq = [rnd.randint(0, 20) for _ in range(rnd.randint(3, 12))]
    k = rnd.randint(1, len(seq))
    blocks = blockpartition.solve(seq, k)
    assert len(blocks) == k and all(blocks)
    assert [x for b in blocks for x in b] == seq
    assert max(sum(b) for b in blocks) == _brute_force_minmax(seq, k)


def test_balance_by_time():
    class Delay(nn.Module):
        def __init__(self, seconds):
            super().__init__()
            self.seconds = seconds

        def forward(self, x):
            time.sleep(self.seconds)
            return x

    model = nn.Sequential(*[Delay(i / 100) for i in [1, 2, 3, 4, 5, 6]])
    assert balance_by_time(2, model, torch.rand(1), device='cpu') == [4, 2]


def test_balance_by_time_loop_resets_input():
    # A layer changing the input shape must not break the next profiling loop.
    class Flatten(nn.Module):
        def forward(self, x):
            return x.flatten(1)

    model = nn.Sequential(nn.Conv2d(3, 2, 1), Flatten(), nn.Linear(128, 10))
    sample = torch.rand(10, 3, 8, 8)
    assert balance_by_time(2, model, sample, device='cpu') in ([1, 2], [2, 1])


def test_balance_by_time_requires_no_grad_yet():
    model = nn.Sequential(nn.Linear(1, 1), nn.Linear(1, 1))
    model(torch.rand(1, 1)).sum().backward()
    with pytest.raises(ValueError, match='some parameter already has gradient'):
        balance_by_time(2, model, torch.rand(1, 1), device='cpu')


def test_balance_by_size_requires_gpu():
    model = nn.Sequential(nn.Linear(1, 1))
    with pytest.raises(ValueError, match='size profiler supports only CUDA device'):
        balance_by_size(1, model, torch.rand(1, 1), device='cpu')


@gpu
def test_balance_by_size_latent():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')

    class Expand(nn.Module):
        def __init__(self, times):
            super().__init__()
            self.times = times

        def forward(self, x):
            for _ in range(self.times):
                x = x + torch.rand_like(x, requires_grad=True)
            return x

    sample = torch.rand(10, 100, 100)
    model = nn.Sequential(*[Expand(i) for i in [1, 2, 3, 4, 5, 6]])
    assert balance_by_size(2, model, sample) == [4, 2]
    model = nn.Sequential(*[Expand(i) for i in [6, 5, 4, 3, 2, 1]])
    assert balance_by_size(2, model, sample) == [2, 4]


@gpu
def test_balance_by_size_param():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    model = nn.Sequential(*[nn.Linear(i + 1, i + 2) for i in range(6)])
    sample = torch.rand(7, 1)
    assert balance_by_size(2, model, sample, param_scale=100) == [4, 2]
    model = nn.Sequential(*[nn.Linear(i + 2, i + 1) for i in reversed(range(6))])
    sample = torch.rand(1, 7)
    assert balance_by_size(2, model, sample, param_scale=100) == [2, 4]


def test_sandbox():
    model = nn.Sequential(nn.BatchNorm2d(3))
    before = {k: v.clone() for k, v in model.state_dict().items()}
    sample = torch.rand(1, 3, 10, 10)
    balance_by_time(1, model, sample, device='cpu')
    after = model.state_dict()
    assert before.keys() == after.keys()
    for key, value in before.items():
        assert torch.allclose(after[key], value), key


def test_not_training():
    class AssertTraining(nn.Module):
        def forward(self, x):
            assert self.training
            return x

    model = nn.Sequential(AssertTraining())
    model.eval()
    assert not model.training
    balance_by_time(1, model, torch.rand(1), device='cpu')
    assert not model.training


def test_sandbox_during_profiling():
    model = nn.Sequential(nn.Linear(1, 1))
    copies = list(layerwise_sandbox(model, torch.device('cpu')))
    assert copies[0] is not model[0]
    assert copies[0].weight is not model[0].weight


def test_deprecated_torchgpipe_amd_balancing():
    with pytest.raises(ImportError, match="import 'torchgpipe_amd.balance' instead"):
        __import__('torchgpipe_amd_balancing')


class _Twin(nn.Module):
    def forward(self, x):
        return x, x.detach()


class _Add(nn.Module):
    def forward(self, pair):
        a, b = pair
        return a + b


def test_balance_by_time_tuple_boundaries():
    model = nn.Sequential(_Twin(), _Add())
    assert balance_by_time(1, model, torch.rand(1, requires_grad=True), device='cpu') == [2]


@gpu
def test_balance_by_size_tuple_boundaries():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    model = nn.Sequential(_Twin(), _Add())
    assert balance_by_size(1, model, torch.rand(1, requires_grad=True)) == [2]


@gpu
def test_balance_by_size_param_scale_tradeoff():
    """param_scale weighs parameters against activations: with no weight the
    activation-heavy front layers dominate, with a heavy weight the
    parameter-heavy back layers do."""
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')

    class Tradeoff(nn.Module):
        def __init__(self, params, latents):
            super().__init__()
            self.fc = nn.Linear(params, params)
            self.latents = latents

        def forward(self, x):
            for _ in range(self.latents):
                x = x + torch.rand_like(x, requires_grad=True)
            return x

    model = nn.Sequential(*[Tradeoff(p, 7 - p) for p in range(1, 7)])
    sample = torch.rand(1, requires_grad=True)
    assert balance_by_size(2, model, sample, param_scale=0) == [2, 4]
    assert balance_by_size(2, model, sample, param_scale=100) == [4, 2]


def test_balance_from_layers_script(tmp_path):
    """scripts/balance_from_layers.py: min-max partition of a per-layer stage profile and
    the GPipe-bubble throughput prediction, for the tuned and a reference balance."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    times = [4.0, 1.0, 1.0, 1.0, 1.0, 4.0]
    prof = {'stages': [{'stage': i, 'layers': [i, i + 1], 'device_ms': t}
                       for i, t in enumerate(times)]}
    path = tmp_path / 'profile.json'
    path.write_text(json.dumps(prof))
    out = subprocess.run([sys.executable, os.path.join(root, 'scripts', 'balance_from_layers.py'),
                          str(path), '--parts', '2', '3', '--batch', '64', '--chunks', '4',
                          '--ref', '3,3', '--scale', '2'],
                         check=True, capture_output=True, text=True).stdout
    rows = [json.loads(line) for line in out.splitlines()]
    tuned2 = next(r for r in rows if r['parts'] == 2 and r['balance_source'] == 'tuned')
    assert tuned2['balance'] == [3, 3] and tuned2['max_stage_ms'] == 12.0
    # bubble: max stage x (m + n - 1) / m = 12 ms x 5 / 4
    assert tuned2['predicted_samples_per_sec'] == round(64 / 0.015, 1)
    tuned3 = next(r for r in rows if r['parts'] == 3)
    assert max(tuned3['stage_ms']) == 8.0
    assert any(r['balance_source'] == 'ref' and r['balance'] == [3, 3] for r in rows)
