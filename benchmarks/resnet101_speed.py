"""ResNet-101 speed benchmark (reference: benchmarks/resnet101-speed/main.py:22-67).

    python benchmarks/resnet101_speed.py pipeline-2 --devices 0,1
"""
import torch
import torch.nn.functional as F

from common import parser, run_speed

from torchgpipe_amd.models import resnet101

EXPERIMENTS = {
    'baseline': dict(batch=118),
    'pipeline-1': dict(batch=220, chunks=2, balance=[370]),
    'pipeline-2': dict(batch=25000, chunks=1667, balance=[135, 235]),
    'pipeline-4': dict(batch=5632, chunks=256, balance=[44, 92, 124, 110]),
    'pipeline-8': dict(batch=5400, chunks=150, balance=[26, 22, 33, 44, 44, 66, 66, 69]),
    # the minimum end-to-end slice of SURVEY §7.3
    'pipeline-2-m32': dict(batch=256, chunks=32, balance=[135, 235], checkpoint='always'),
}


def main() -> None:
    args = parser(__doc__, EXPERIMENTS).parse_args()
    run_speed(args, EXPERIMENTS[args.experiment], lambda: resnet101(num_classes=1000),
              (3, 224, 224), lambda b, d: torch.randint(1000, (b,), device=d),
              F.cross_entropy, dataset_size=50000)


if __name__ == '__main__':
    main()
