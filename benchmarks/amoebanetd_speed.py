"""AmoebaNet-D(18,256) speed benchmark (reference: benchmarks/amoebanetd-speed/main.py:35-96).

Checkpointing is 'always' for m=1 and 'except_last' otherwise.

    python benchmarks/amoebanetd_speed.py n8m32 --devices 0,1,2,3,4,5,6,7
"""
import torch
import torch.nn.functional as F

from common import parser, run_speed

from torchgpipe_amd.models import amoebanetd


def exp(batch, chunks, balance):
    return dict(batch=batch, chunks=chunks, balance=balance,
                checkpoint='always' if chunks == 1 else 'except_last')


EXPERIMENTS = {
    'n2m1': exp(96, 1, [7, 17]),
    'n2m4': exp(256, 4, [9, 15]),
    'n2m32': exp(1280, 32, [9, 15]),
    'n4m1': exp(160, 1, [3, 4, 5, 12]),
    'n4m4': exp(360, 4, [3, 6, 7, 8]),
    'n4m32': exp(1152, 32, [3, 6, 7, 8]),
    'n8m1': exp(196, 1, [2, 2, 2, 2, 2, 3, 4, 7]),
    'n8m4': exp(480, 4, [2, 2, 2, 3, 3, 4, 4, 4]),
    'n8m32': exp(1280, 32, [2, 2, 2, 3, 3, 4, 4, 4]),
}


def main() -> None:
    args = parser(__doc__, EXPERIMENTS).parse_args()
    run_speed(args, EXPERIMENTS[args.experiment],
              lambda: amoebanetd(num_classes=1000, num_layers=18, num_filters=256),
              (3, 224, 224), lambda b, d: torch.randint(1000, (b,), device=d),
              F.cross_entropy, dataset_size=10000)


if __name__ == '__main__':
    main()
