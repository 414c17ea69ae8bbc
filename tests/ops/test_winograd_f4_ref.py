"""CPU check of the F(4x4,3x3) Winograd algebra used by csrc/winograd_f4.hip.

Emulates the kernel's data flow in float64 (same B^T / G / A^T matrices, the same
6x6 patch origin (4ty-1, 4tx-1), zero padding taps, partial edge tiles) and compares
with F.conv2d, so a wrong coefficient or tile convention fails here, not on the GPU.
"""
import pytest
import torch
import torch.nn.functional as F

BT = torch.tensor([[4, 0, -5, 0, 1, 0],
                   [0, -4, -4, 1, 1, 0],
                   [0, 4, -4, -1, 1, 0],
                   [0, -2, -1, 2, 1, 0],
                   [0, 2, -1, -2, 1, 0],
                   [0, 4, 0, -5, 0, 1]], dtype=torch.float64)
G = torch.tensor([[1 / 4, 0, 0],
                  [-1 / 6, -1 / 6, -1 / 6],
                  [-1 / 6, 1 / 6, -1 / 6],
                  [1 / 24, 1 / 12, 1 / 6],
                  [1 / 24, -1 / 12, 1 / 6],
                  [0, 0, 1]], dtype=torch.float64)
AT = torch.tensor([[1, 1, 1, 1, 1, 0],
                   [0, 1, -1, 2, -2, 0],
                   [0, 1, 1, 4, 4, 0],
                   [0, 1, -1, 8, -8, 1]], dtype=torch.float64)


def f4_conv(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    n, c, h, wd = x.shape
    k = w.shape[0]
    th, tw = (h + 3) // 4, (wd + 3) // 4
    # pad so every 6x6 patch starting at (4ty-1, 4tx-1) is inside the padded image
    xp = F.pad(x, (1, 4 * tw + 1 - wd, 1, 4 * th + 1 - h))
    d = xp.unfold(2, 6, 4).unfold(3, 6, 4)                    # n c th tw 6 6
    v = torch.einsum('ia,nctwab,jb->nctwij', BT, d, BT)       # B^T d B
    u = torch.einsum('ia,kcab,jb->kcij', G, w, G)             # G g G^T
    m = torch.einsum('kcij,nctwij->nktwij', u, v)             # 36 GEMMs over c
    y = torch.einsum('pi,nktwij,qj->nktwpq', AT, m, AT)       # A^T M A
    y = y.permute(0, 1, 2, 4, 3, 5).reshape(n, k, 4 * th, 4 * tw)
    return y[:, :, :h, :wd]


@pytest.mark.parametrize('shape', [(2, 3, 5, 8, 8), (1, 4, 2, 12, 12), (2, 2, 3, 7, 10),
                                   (1, 5, 4, 1, 6), (1, 1, 1, 13, 5)])
def test_f4_algebra_matches_conv2d(shape):
    n, c, k, h, w = shape
    torch.manual_seed(0)
    x = torch.randn(n, c, h, w, dtype=torch.float64)
    wt = torch.randn(k, c, 3, 3, dtype=torch.float64)
    torch.testing.assert_close(f4_conv(x, wt), F.conv2d(x, wt, padding=1), rtol=1e-10, atol=1e-10)


def test_f4_backward_data_is_flipped_transposed_forward():
    # the kernel runs backward-data as the forward convolution with w rotated 180 degrees
    # and in/out channels swapped (the weight transform's `flip`)
    torch.manual_seed(1)
    x = torch.randn(2, 3, 9, 11, dtype=torch.float64, requires_grad=True)
    wt = torch.randn(5, 3, 3, 3, dtype=torch.float64)
    y = F.conv2d(x, wt, padding=1)
    dy = torch.randn_like(y)
    y.backward(dy)
    flipped = wt.flip(2, 3).transpose(0, 1).contiguous()
    torch.testing.assert_close(f4_conv(dy, flipped), x.grad, rtol=1e-10, atol=1e-10)
