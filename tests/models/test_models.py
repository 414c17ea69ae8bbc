import pytest
import torch

from torchgpipe_amd.models import amoebanetd, resnet101, unet
from torchgpipe_amd.skip import verify_skippables


def n_params(m):
    return sum(p.numel() for p in m.parameters())


def test_unet_5_64_matches_reference_layout():
    m = unet(depth=5, num_convs=5, base_channels=64)
    assert len(m) == 241
    assert n_params(m) == 232_687_328
    verify_skippables(m)
    names = [n for n, _ in m.named_children()]
    assert names[:4] == ['encoder_0_encode_0_conv', 'encoder_0_encode_0_dropout',
                         'encoder_0_encode_0_norm', 'encoder_0_encode_0_relu']
    assert names[-1] == 'segment'


def test_unet_fused_equals_unfused_in_eval():
    torch.manual_seed(0)
    fused = unet(depth=2, num_convs=2, base_channels=8, fused=True)
    plain = unet(depth=2, num_convs=2, base_channels=8, fused=False)
    plain.load_state_dict(fused.state_dict())
    fused.eval()
    plain.eval()
    x = torch.rand(2, 3, 32, 32)
    torch.testing.assert_close(fused(x), plain(x), rtol=1e-4, atol=1e-5)


def test_unet_state_dict_identical_fused_unfused():
    assert unet(depth=2, base_channels=8).state_dict().keys() == \
        unet(depth=2, base_channels=8, fused=False).state_dict().keys()


def test_amoebanetd_18_256():
    m = amoebanetd(num_classes=1000, num_layers=18, num_filters=256)
    assert len(m) == 24
    assert n_params(m) == 122_470_120


def test_amoebanetd_small_forward_backward():
    m = amoebanetd(num_classes=10, num_layers=3, num_filters=32)
    y = m(torch.rand(2, 3, 224, 224))
    assert y.shape == (2, 10)
    y.sum().backward()


def test_resnet101():
    m = resnet101()
    assert len(m) == 370
    assert n_params(m) == 44_549_160
    verify_skippables(m)


@pytest.mark.parametrize('depth', [1, 2, 3])
def test_unet_depths_run(depth):
    m = unet(depth=depth, num_convs=1, base_channels=4)
    y = m(torch.rand(1, 3, 16, 16))
    assert y.shape == (1, 1, 16, 16)
