"""The distributed accuracy driver trains through DistributedGPipe on 2 gloo ranks."""
import math
import os
import sys

from tests.distributed.mp_util import run

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', '..', 'benchmarks'))


def _worker(rank, world):
    import distributed_accuracy as acc
    args = acc.parse(['naive-128', '--model', 'mlp-tiny', '--balance', '3,3', '--chunks', '4',
                      '--batch-size', '32', '--epochs', '3', '--skip-epochs', '1',
                      '--image-size', '16', '--synthetic-size', '640', '--lr', '0.02',
                      '--device', 'cpu'])
    return acc.train(args)


def test_distributed_accuracy_driver_learns_on_gloo(tmp_path):
    results = run(_worker, 2, tmp_path)
    last = results[-1]
    assert math.isfinite(last['samples_per_sec']) and last['samples_per_sec'] > 0
    # the synthetic classes are separable: well above chance (0.1) after 3 epochs
    assert last['accuracy'] > 0.5, last


def test_lr_schedule_matches_reference_recipe():
    import distributed_accuracy as acc
    assert acc.lr_multiplier(0, 100, 128) == 1.0
    assert acc.lr_multiplier(200, 100, 1024) == 2.5  # half-way through the 4-epoch warm-up
    assert abs(acc.lr_multiplier(3100, 100, 256) - 0.1) < 1e-12
