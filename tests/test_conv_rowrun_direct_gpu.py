"""Few-channel first-layer direct kernels (conv_rowrun_direct.hip: AlexNet conv1, 3 channels on
228-pixel rows, 11 x 11 / 4, 96 outputs; GoogLeNet conv1, 4-channel NHWC 224 x 224, 7 x 7 / 2,
pad 3, 64 outputs -- padding staged on the fly) against fp32 torch.  Weight gradient: the 1-GPU batch,
the 8-GPU strong-scaling batch, odd image counts, a map whose last row group is short (14 output
rows = 3 groups of 4 + 2), a channel-sliced dy, accumulation into dw, bitwise repeatability and
the shapes it must refuse.  Forward: the same batches and maps, bias / relu, an output channel
slice of a wider buffer (nothing outside it written), and the conv_forward dispatch."""
import torch.nn.functional as F
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


@pytest.mark.parametrize("N,H,ldc,relu,bias", [(256, 227, 96, True, True), (32, 227, 96, False, True),
                                               (3, 227, 96, True, False), (5, 63, 96, True, True),
                                               (2, 63, 128, False, True)])
def test_rowrun_fwd2(N, H, ldc, relu, bias):
    from cxxnet_amd import native
    g = _geo(N, H)
    x = _rnd((N, H, 228, 3), 7)
    w = (_rnd((96, 11, 11, 3), 8).float() * 0.05).to(torch.bfloat16)
    b = torch.randn(96, device=DEV) if bias else None
    yb = torch.full((N, g.Ho, 55, ldc), 7.0, device=DEV, dtype=torch.bfloat16)
    y = yb[..., :96]
    rc = native.kernels().cxn_conv_rowrun_fwd2(x.data_ptr(), w.data_ptr(), b.data_ptr() if bias else None, y.data_ptr(),
                                               N, H, 228, 3, g.Ho, 55, 96, ldc, 11, 11, 4, 0, int(relu),
                                               torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, stride=4)
    if relu:
        ref = ref.clamp_min(0)
    got = y.float().permute(0, 3, 1, 2)
    assert ((got - ref).norm() / ref.norm()).item() < 5e-3
    if ldc > 96:
        assert torch.all(yb[..., 96:] == 7.0)  # nothing outside the slice


def test_rowrun_fwd2_through_conv_forward():
    g = _geo(4, 227)
    x = _rnd((4, 227, 228, 3), 9)
    w = (_rnd((96, 11, 11, 3), 10).float() * 0.05).to(torch.bfloat16)
    b = torch.randn(96, device=DEV)
    y = torch.empty((4, 55, 55, 96), device=DEV, dtype=torch.bfloat16)
    gemm.conv_forward(x, w, b, y, g, relu=True)
    torch.cuda.synchronize()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, stride=4).clamp_min(0)
    assert ((y.float().permute(0, 3, 1, 2) - ref).norm() / ref.norm()).item() < 5e-3


def _ggeo(N, H=224):
    Ho = (H + 6 - 7) // 2 + 1
    return ConvGeom(N, H, 224, 4, Ho, 112, 64, 7, 7, 2, 3, 3, 1)


@pytest.mark.parametrize("N,H", [(128, 224), (32, 224), (3, 224), (2, 20)])
def test_rowrun_googlenet_wgrad(N, H):
    g = _ggeo(N, H)
    x = _rnd((N, H, 224, 4), 21)
    dy = _rnd((N, g.Ho, 112, 64), 22)
    dw = torch.full((64, 7, 7, 4), 0.25, device=DEV)
    assert gemm.conv_wgrad_rowrun(x, dy, dw, g)
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (64, 4, 7, 7), dy.float().permute(0, 3, 1, 2),
                                      stride=2, padding=3)
    err = (((dw - 0.25).permute(0, 3, 1, 2) - ref).norm() / ref.norm()).item()
    assert err < 1e-5, err
    dw2 = torch.full_like(dw, 0.25)
    assert gemm.conv_wgrad_rowrun(x, dy, dw2, g)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw2)


@pytest.mark.parametrize("N,H,relu", [(128, 224, True), (32, 224, False), (3, 224, True), (2, 20, True)])
def test_rowrun_googlenet_fwd(N, H, relu):
    g = _ggeo(N, H)
    x = _rnd((N, H, 224, 4), 23)
    w = (_rnd((64, 7, 7, 4), 24).float() * 0.05).to(torch.bfloat16)
    b = torch.randn(64, device=DEV)
    y = torch.full((N, g.Ho, 112, 64), 7.0, device=DEV, dtype=torch.bfloat16)
    assert gemm.conv_rowrun_fwd2(x, w, b, y, g, relu=relu)
    torch.cuda.synchronize()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, stride=2, padding=3)
    if relu:
        ref = ref.clamp_min(0)
    assert ((y.float().permute(0, 3, 1, 2) - ref).norm() / ref.norm()).item() < 5e-3
