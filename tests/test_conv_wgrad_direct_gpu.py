"""Direct small-map weight gradient (csrc/kernels/conv_wgrad_direct.hip) against fp32 torch:
AlexNet's 13 x 13 layers (conv3 256->384, grouped conv4 / conv5), 14 x 14 (VGG-16 conv5_x,
GoogLeNet 4c / 4e), an odd image count (the last
stage holds one image: the missing one must read as zeros), forced split counts, a dy channel
slice, accumulation into a non-zero dW (+=), and bitwise reproducibility."""
import pytest
import torch

from cxxnet_amd.ops import gemm
from cxxnet_amd.ops.gemm import ConvGeom

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (N, C, Cout, groups, splits)
CASES = [
    (4, 256, 384, 1, 0),   # AlexNet conv3
    (5, 384, 384, 2, 0),   # conv4 (grouped), odd N
    (3, 384, 256, 2, 0),   # conv5 (grouped), odd N
    (7, 64, 64, 1, 3),     # one channel pair, forced splits over 4 stages
    (2, 32, 128, 1, 1),    # two co blocks, one split
    (32, 256, 384, 1, 0),  # the per-GPU batch of 8-GPU strong scaling
    (4, 64, 192, 1, 2),    # three co blocks, 2 ci blocks: bias K-steps k % 2 per ci block
    (64, 512, 512, 1, 0, 14),  # VGG-16 conv5_x: 14 x 14, one image per stage
    (5, 128, 256, 1, 0, 14),   # GoogLeNet inception 4c's 3 x 3, odd N
    (3, 160, 320, 1, 2, 14),   # GoogLeNet 4e, forced splits
]


def _rnd(shape, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(*shape, generator=g, device=DEV).to(torch.bfloat16)


def _ref(x, dy, groups):
    C, Cout = x.shape[3], dy.shape[3]
    return torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (Cout, C // groups, 3, 3),
                                       dy.float().permute(0, 3, 1, 2), stride=1, padding=1, groups=groups)


def _err(got, ref):
    return ((got - ref).norm() / ref.norm()).item()


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_wgrad_direct(case):
    N, C, Cout, groups, splits = case[:5]
    H = case[5] if len(case) > 5 else 13
    g = ConvGeom(N, H, H, C, H, H, Cout, 3, 3, 1, 1, 1, groups)
    x = _rnd((N, H, H, C), 1)
    dy = _rnd((N, H, H, Cout), 2)
    dw = torch.full((Cout, 3, 3, C // groups), 0.5, device=DEV)
    db = torch.full((Cout,), 0.25, device=DEV)
    assert gemm.conv_wgrad_direct(x, dy, dw, g, splits=splits, db=db)
    torch.cuda.synchronize()
    got = (dw - 0.5).permute(0, 3, 1, 2)
    err = _err(got, _ref(x, dy, groups))
    assert err < 1e-5, err  # fp32 accumulation of bf16 products: only the summation order differs
    dbref = dy.float().sum((0, 1, 2))
    assert _err(db - 0.25, dbref) < 1e-5
    dw2 = torch.full_like(dw, 0.5)
    db2 = torch.full_like(db, 0.25)
    assert gemm.conv_wgrad_direct(x, dy, dw2, g, splits=splits, db=db2)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw2) and torch.equal(db, db2)  # fixed split order, no atomics
    dw3 = torch.full_like(dw, 0.5)
    assert gemm.conv_wgrad_direct(x, dy, dw3, g, splits=splits)  # without the bias: same dW
    torch.cuda.synchronize()
    assert torch.equal(dw, dw3)


def test_wgrad_direct_dy_slice_and_accumulate():
    N, C, Cout = 3, 128, 128
    g = ConvGeom(N, 13, 13, C, 13, 13, Cout, 3, 3, 1, 1, 1, 1)
    x = _rnd((N, 13, 13, C), 3)
    big = _rnd((N, 13, 13, Cout + 64), 4)
    dy = big[..., 64:]  # a channel slice: pixel stride 192
    dw = torch.zeros((Cout, 3, 3, C), device=DEV)
    assert gemm.conv_wgrad_direct(x, dy, dw, g)
    assert gemm.conv_wgrad_direct(x, dy, dw, g)  # += : twice the gradient
    torch.cuda.synchronize()
    ref = _ref(x, dy.contiguous(), 1)
    assert _err(dw.permute(0, 3, 1, 2), 2 * ref) < 1e-5


def test_wgrad_direct_declines_unserved_shapes():
    x = _rnd((2, 12, 12, 64), 5)  # (13 x 13 and 14 x 14 are served, 12 x 12 is not)
    dy = _rnd((2, 12, 12, 64), 6)
    dw = torch.zeros((64, 3, 3, 64), device=DEV)
    assert not gemm.conv_wgrad_direct(x, dy, dw, ConvGeom(2, 12, 12, 64, 12, 12, 64, 3, 3, 1, 1, 1, 1))
    x = _rnd((2, 13, 13, 48), 5)
    dy = _rnd((2, 13, 13, 64), 6)
    dw = torch.zeros((64, 3, 3, 48), device=DEV)
    assert not gemm.conv_wgrad_direct(x, dy, dw, ConvGeom(2, 13, 13, 48, 13, 13, 64, 3, 3, 1, 1, 1, 1))


# AlexNet conv2 (27 x 27, 5 x 5, 48 input / 128 output channels per group): the tap-split form,
# two 14 / 13-row bands per image, no bias gradient (conv2's comes from the pool behind it)
CASES5 = [
    (256, 96, 256, 2, 0),
    (32, 96, 256, 2, 0),
    (3, 48, 64, 1, 0),    # odd N, one channel pair
    (5, 32, 128, 1, 3),   # two input-channel units, forced splits
]


@pytest.mark.parametrize("case", CASES5, ids=lambda c: "x".join(map(str, c)))
def test_wgrad_direct_5x5_bands(case):
    N, C, Cout, groups, splits = case
    g = ConvGeom(N, 27, 27, C, 27, 27, Cout, 5, 5, 1, 2, 2, groups)
    x = _rnd((N, 27, 27, C), 11)
    dy = _rnd((N, 27, 27, Cout), 12)
    dw = torch.full((Cout, 5, 5, C // groups), 0.5, device=DEV)
    assert gemm.conv_wgrad_direct(x, dy, dw, g, splits=splits)
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (Cout, C // groups, 5, 5),
                                      dy.float().permute(0, 3, 1, 2), stride=1, padding=2, groups=groups)
    err = _err((dw - 0.5).permute(0, 3, 1, 2), ref)
    assert err < 1e-5, err
    dw2 = torch.full_like(dw, 0.5)
    assert gemm.conv_wgrad_direct(x, dy, dw2, g, splits=splits)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw2)  # fixed split order, no atomics
    db = torch.zeros(Cout, device=DEV)
    assert not gemm.conv_wgrad_direct(x, dy, dw2, g, splits=splits, db=db)  # no bias-gradient form: not served
