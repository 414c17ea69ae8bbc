"""Timing probe: would forward lanes pay on ResNet-101's small-micro-batch stages?

PipelineStage keeps a partition with running statistics (BatchNorm) on one stream.  This
runs benchmarks/stage_harness.py with every BatchNorm's running statistics off
(track_running_stats=False: the same batch-statistics compute, no running update), so the
stage is eligible for forward lanes, and ``--lanes on|off`` times it with and without.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..',
                                'benchmarks'))

import torch  # noqa: E402

import stage_harness  # noqa: E402

_build = stage_harness.build


def build(kind, dev):
    model = _build(kind, dev)
    for m in model.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            m.track_running_stats = False
            m.running_mean = m.running_var = m.num_batches_tracked = None
    return model


stage_harness.build = build

if __name__ == '__main__':
    stage_harness.main()
