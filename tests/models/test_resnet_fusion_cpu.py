"""Layer fusion links of the ResNet model (ops/fusion.py) on the CPU: the fused layers fall
back to their plain forward and compute the plain model's function."""
import torch
from torch import nn

from torchgpipe_amd.models.resnet import build_resnet
from torchgpipe_amd.ops.fusion import BatchNormAct2d, ConvBN2d, ReLU, relink


def test_links_stay_inside_a_partition():
    model = build_resnet([1, 1, 1, 1], num_classes=10)
    layers = list(model.children())
    # conv1, bn1, relu, maxpool, then the first bottleneck
    assert relink(model) == 1 + 4 * 3 + 4  # stem + 3 per block + 4 downsamples
    first = nn.Sequential(*layers[:6])      # ... identity, conv1 of block 1 (its bn1 not)
    assert relink(first) == 1                # only the stem keeps its link
    assert '_tgpipe_link' not in layers[5].__dict__
    assert '_tgpipe_link' in layers[0].__dict__


def test_fused_model_equals_plain_model_on_cpu():
    torch.manual_seed(0)
    fused = build_resnet([1, 1, 1, 1], num_classes=10, fused=True)
    plain = build_resnet([1, 1, 1, 1], num_classes=10, fused=False)
    assert list(fused.state_dict()) == list(plain.state_dict())
    plain.load_state_dict(fused.state_dict())
    x = torch.randn(2, 3, 64, 64)
    torch.testing.assert_close(fused(x), plain(x))
    fused.eval()
    plain.eval()
    torch.testing.assert_close(fused(x), plain(x))


def test_fused_layers_are_nn_subclasses():
    assert issubclass(ConvBN2d, nn.Conv2d)
    assert issubclass(BatchNormAct2d, nn.BatchNorm2d)
    assert issubclass(ReLU, nn.ReLU)


def test_conv3_is_linked_to_its_residual_join():
    """conv3, bn3, residual, relu3: conv3's link names the residual join that runs it
    (ops/fusion.py pending_join); conv1 / conv2 link to their BatchNorm + ReLU only."""
    model = build_resnet([1, 1, 1, 1], num_classes=10)
    layers = list(model.children())
    conv1, conv3, residual = layers[5], layers[11], layers[13]
    assert conv1.__dict__['_tgpipe_link'][1:] == (True, None)
    bn, relu, join = conv3.__dict__['_tgpipe_link']
    assert bn is layers[12] and relu is False
    assert join is getattr(residual, 'module', residual)
    # split after bn3: the join is in another partition, conv3 keeps a plain BN link
    relink(nn.Sequential(*layers[:13]))
    assert conv3.__dict__['_tgpipe_link'][2] is None
