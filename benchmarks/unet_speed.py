"""U-Net(5,64) speed benchmark (reference: benchmarks/unet-speed/main.py:23-68).

    python benchmarks/unet_speed.py pipeline-8 --devices 0,1,2,3,4,5,6,7
    python -m torch.distributed.run --nproc-per-node 8 benchmarks/unet_speed.py pipeline-8 \\
        --mode stage
"""
import torch
import torch.nn.functional as F

from common import parser, run_speed

from torchgpipe_amd.models import unet

EXPERIMENTS = {
    'baseline': dict(batch=40),
    'pipeline-1': dict(batch=80, chunks=2, balance=[241]),
    'pipeline-2': dict(batch=512, chunks=32, balance=[104, 137]),
    'pipeline-4': dict(batch=512, chunks=16, balance=[30, 66, 84, 61]),
    'pipeline-8': dict(batch=640, chunks=40, balance=[16, 27, 31, 44, 22, 57, 27, 17]),
    # MI355X-tuned balances (see bench.py / profiles/unet_layer_profile.json)
    'pipeline-2-tuned': dict(batch=512, chunks=32, balance=[97, 144]),
    'pipeline-4-tuned': dict(batch=512, chunks=16, balance=[39, 54, 58, 90]),
    'pipeline-8-tuned': dict(batch=640, chunks=40, balance=[18, 27, 29, 23, 25, 33, 44, 42]),
}


def main() -> None:
    args = parser(__doc__, EXPERIMENTS).parse_args()
    run_speed(args, EXPERIMENTS[args.experiment],
              lambda: unet(depth=5, num_convs=5, base_channels=64, input_channels=3,
                           output_channels=1),
              (3, 192, 192), lambda b, d: torch.ones(b, 1, 192, 192, device=d),
              F.binary_cross_entropy_with_logits, dataset_size=10000)


if __name__ == '__main__':
    main()
