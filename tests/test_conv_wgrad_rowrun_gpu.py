"""Few-channel first-layer weight gradient (conv_wgrad_direct.hip conv_wgrad_rowrun: AlexNet
conv1, 3 channels on 228-pixel rows, 11 x 11 / 4, 96 outputs) against fp32 torch: the 1-GPU batch,
the 8-GPU strong-scaling batch, odd image counts, a map whose last row group is short (14 output
rows = 3 groups of 4 + 2), a channel-sliced dy, accumulation into dw, bitwise repeatability and
the shapes it must refuse."""
import pytest
import torch

from cxxnet_amd.ops import gemm
from cxxnet_amd.ops.gemm import ConvGeom

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rnd(shape, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(*shape, generator=g, device=DEV).to(torch.bfloat16)


def _geo(N, H):
    Ho = (H - 11) // 4 + 1
    return ConvGeom(N, H, 228, 3, Ho, 55, 96, 11, 11, 4, 0, 0, 1)


@pytest.mark.parametrize("N,H,ldy", [(256, 227, 96), (32, 227, 96), (3, 227, 96), (5, 63, 96), (2, 63, 128)])
def test_rowrun_wgrad(N, H, ldy):
    g = _geo(N, H)
    x = _rnd((N, H, 228, 3), 1)
    dyb = _rnd((N, g.Ho, 55, ldy), 2)
    dy = dyb[..., :96]
    dw = torch.full((96, 11, 11, 3), 0.25, device=DEV)
    assert gemm.conv_wgrad_rowrun(x, dy, dw, g)
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (96, 3, 11, 11), dy.float().permute(0, 3, 1, 2),
                                      stride=4)
    got = (dw - 0.25).permute(0, 3, 1, 2)
    err = ((got - ref).norm() / ref.norm()).item()
    assert err < 1e-5, err
    dw2 = torch.full_like(dw, 0.25)
    assert gemm.conv_wgrad_rowrun(x, dy, dw2, g)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw2)  # fixed-order partial sums


def test_rowrun_wgrad_through_backward_weight():
    """conv_backward_weight picks the direct kernel for the conv1 shape (and leaves db to the caller)."""
    g = _geo(4, 227)
    x = _rnd((4, 227, 228, 3), 3)
    dy = _rnd((4, 55, 55, 96), 4)
    dw = torch.zeros((96, 11, 11, 3), device=DEV)
    db = torch.zeros(96, device=DEV)
    assert gemm.conv_backward_weight(x, dy, dw, g, db=db) is False
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (96, 3, 11, 11), dy.float().permute(0, 3, 1, 2),
                                      stride=4)
    assert ((dw.permute(0, 3, 1, 2) - ref).norm() / ref.norm()).item() < 1e-5


@pytest.mark.parametrize("change", ["stride", "cout", "width", "pad"])
def test_rowrun_wgrad_refuses(change):
    N, H = 2, 63
    kw = dict(N=N, H=H, W=228, C=3, Ho=14, Wo=55, Cout=96, KH=11, KW=11, stride=4, pad_y=0, pad_x=0, groups=1)
    if change == "stride":
        kw.update(stride=2, Ho=27, Wo=109)
    elif change == "cout":
        kw.update(Cout=64)
    elif change == "width":
        kw.update(W=224, Wo=54)
    else:
        kw.update(pad_y=1, pad_x=1)
    g = ConvGeom(kw["N"], kw["H"], kw["W"], kw["C"], kw["Ho"], kw["Wo"], kw["Cout"], kw["KH"], kw["KW"], kw["stride"],
                 kw["pad_y"], kw["pad_x"], kw["groups"])
    x = _rnd((N, H, kw["W"], 3), 5)
    dy = _rnd((N, kw["Ho"], kw["Wo"], kw["Cout"]), 6)
    dw = torch.zeros((kw["Cout"], 11, 11, 3), device=DEV)
    assert not gemm.conv_wgrad_rowrun(x, dy, dw, g)
