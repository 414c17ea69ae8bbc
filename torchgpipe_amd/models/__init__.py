"""Benchmark model zoo: flat ``nn.Sequential`` builders matching the reference benchmarks."""
from torchgpipe_amd.models.amoebanet import amoebanetd
from torchgpipe_amd.models.resnet import resnet101
from torchgpipe_amd.models.unet import unet

__all__ = ['unet', 'amoebanetd', 'resnet101']
