"""ResNet-101 speed benchmark (reference: benchmarks/resnet101-speed/main.py:22-67).

    python benchmarks/resnet101_speed.py pipeline-2 --devices 0,1
"""
import torch
import torch.nn.functional as F

from common import parser, run_speed

from torchgpipe_amd.models.resnet import build_resnet

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
    p = parser(__doc__, EXPERIMENTS)
    p.add_argument('--plain', action='store_true',
                   help='plain nn layers (MIOpen convolutions / BatchNorm) instead of the fused '
                        'Conv-BN-ReLU runs (ops/fusion.py)')
    args = p.parse_args()
    run_speed(args, EXPERIMENTS[args.experiment],
              lambda: build_resnet([3, 4, 23, 3], num_classes=1000, fused=not args.plain),
              (3, 224, 224), lambda b, d: torch.randint(1000, (b,), device=d),
              F.cross_entropy, dataset_size=50000)


if __name__ == '__main__':
    main()
