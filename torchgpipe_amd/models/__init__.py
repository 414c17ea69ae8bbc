"""Benchmark model zoo: flat ``nn.Sequential`` builders matching the reference benchmarks."""
from torchgpipe_amd.models.amoebanet import amoebanetd
from torchgpipe_amd.models.resnet import resnet50, resnet101
from torchgpipe_amd.models.unet import unet
from torchgpipe_amd.models.vgg import vgg16

__all__ = ['unet', 'amoebanetd', 'resnet50', 'resnet101', 'vgg16']
