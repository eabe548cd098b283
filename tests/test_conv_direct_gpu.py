"""Direct small-map forward / data gradient (csrc/kernels/conv_direct.hip) against fp32 torch:
AlexNet's 13 x 13 layers (conv3 256->384, grouped conv4 / conv5) at the 1-GPU batch (256), the
8-GPU strong-scaling batch (32) and odd image counts (the last item holds one image: the missing
one reads as zeros and is not stored), bias + relu, the relu'-masked data gradient with the
bias-gradient sums of the node it writes, and input / output channel slices."""
import pytest
import torch
import torch.nn.functional as F

from cxxnet_amd.ops import gemm
from cxxnet_amd.ops.gemm import ConvGeom

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (N, C, Cout, groups[, H, K]): 13 x 13 / 3 x 3 unless given
CASES = [
    (256, 256, 384, 1),  # AlexNet conv3
    (256, 384, 384, 2),  # conv4
    (256, 384, 256, 2),  # conv5
    (32, 256, 384, 1),   # strong-scaling batch
    (7, 384, 256, 2),    # odd N
    (1, 64, 64, 1),      # one item
    (5, 192, 128, 1),    # six channel stages (data gradient: four)
    (256, 96, 256, 2, 27, 5),  # AlexNet conv2: paired-tap form (forward 48 channels per group, data gradient 128 -> 48)
    (32, 96, 256, 2, 27, 5),
    (3, 64, 128, 1, 27, 5),
    (64, 512, 512, 1, 14, 3),  # VGG-16 conv5_x (14 x 14)
    (5, 128, 256, 1, 14, 3),   # GoogLeNet inception 4c's 3 x 3, odd N
]


def _geo(case):
    N, C, Cout, groups = case[:4]
    H, K = case[4:] if len(case) > 4 else (13, 3)
    return N, C, Cout, groups, H, K


def _rnd(shape, seed, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV) * scale).to(torch.bfloat16)


def _err(got, ref):
    return ((got.float() - ref).norm() / ref.norm()).item()


def _nchw(t):
    return t.float().permute(0, 3, 1, 2)


def _served(variant, C, Cout, groups, H):
    """Version 2 (variant 3) serves channel blocks of 128 / 96 (13 x 13) or 128 / 48 (27 x 27), not
    14 x 14 maps."""
    if variant != 3:
        return True
    if H == 14:
        return False
    cog = Cout // groups
    return cog % 128 == 0 or cog % (96 if H == 13 else 48) == 0


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("variant", [0, 3])
def test_direct_forward(case, relu, variant):
    N, C, Cout, groups, H, K = _geo(case)
    if not _served(variant, C, Cout, groups, H):
        pytest.skip("channel count not served by this variant")
    g = ConvGeom(N, H, H, C, H, H, Cout, K, K, 1, K // 2, K // 2, groups)
    x = _rnd((N, H, H, C), 1)
    w = _rnd((Cout, K, K, C // groups), 2, 0.05)
    b = torch.randn(Cout, device=DEV) * 0.1
    y = torch.full((N, H, H, Cout), 7.0, device=DEV, dtype=torch.bfloat16)
    assert gemm.conv_direct_forward(x, w, b, y, g, relu=relu, variant=variant)
    torch.cuda.synchronize()
    ref = F.conv2d(_nchw(x), w.float().permute(0, 3, 1, 2), b, padding=K // 2, groups=groups)
    if relu:
        ref = ref.clamp_min(0)
    assert _err(y.permute(0, 3, 1, 2), ref) < 5e-3  # bf16 output rounding


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
@pytest.mark.parametrize("mode", ["plain", "mask", "mask_db"])
@pytest.mark.parametrize("variant", [0, 1, 3])
def test_direct_data_grad(case, mode, variant):
    N, C, Cout, groups, H, K = _geo(case)
    if not _served(variant, Cout, C, groups, H):
        pytest.skip("channel count not served by this variant")
    g = ConvGeom(N, H, H, C, H, H, Cout, K, K, 1, K // 2, K // 2, groups)
    dy = _rnd((N, H, H, Cout), 3)
    w = _rnd((Cout, K, K, C // groups), 4, 0.05)
    wt = torch.empty_like(w)
    gemm.conv_weight_flip_multi([(w, wt, g)])
    act = torch.relu(_rnd((N, H, H, C), 5))  # relu(z) of the layer below
    dx = act.clone()
    db = torch.full((C,), 0.5, device=DEV) if mode == "mask_db" else None
    got_db = gemm.conv_direct_data(dy, wt, dx, g, mask_relu=mode != "plain", dbias=db, variant=variant)
    assert got_db
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w.float().permute(0, 3, 1, 2), _nchw(dy), padding=K // 2,
                                     groups=groups)
    if mode != "plain":
        ref = ref * (_nchw(act) > 0).float()
    assert _err(dx.permute(0, 3, 1, 2), ref) < 5e-3
    if db is not None:
        dbref = dx.float().sum((0, 1, 2))  # the column sums of the stored (bf16) dx
        assert _err(db - 0.5, dbref) < 1e-5


def test_direct_channel_slices():
    """x read from a channel slice of a wider buffer and y written into one (zero-copy concat)."""
    N, C, Cout = 3, 128, 128
    g = ConvGeom(N, 13, 13, C, 13, 13, Cout, 3, 3, 1, 1, 1, 1)
    xb = _rnd((N, 13, 13, C + 64), 6)
    x = xb[..., 32:32 + C]
    w = _rnd((Cout, 3, 3, C), 7, 0.05)
    yb = torch.zeros((N, 13, 13, Cout + 64), device=DEV, dtype=torch.bfloat16)
    y = yb[..., 64:]
    assert gemm.conv_direct_forward(x, w, None, y, g)
    torch.cuda.synchronize()
    ref = F.conv2d(_nchw(x.contiguous()), w.float().permute(0, 3, 1, 2), padding=1)
    assert _err(y.permute(0, 3, 1, 2), ref) < 5e-3
    assert torch.count_nonzero(yb[..., :64]) == 0  # nothing outside the slice


def test_direct_data_grad_deterministic():
    N, C, Cout, groups = 32, 384, 256, 2
    g = ConvGeom(N, 13, 13, C, 13, 13, Cout, 3, 3, 1, 1, 1, groups)
    dy = _rnd((N, 13, 13, Cout), 8)
    w = _rnd((Cout, 3, 3, C // groups), 9, 0.05)
    wt = torch.empty_like(w)
    gemm.conv_weight_flip_multi([(w, wt, g)])
    outs = []
    for _ in range(2):
        dx = torch.empty((N, 13, 13, C), device=DEV, dtype=torch.bfloat16)
        assert gemm.conv_direct_data(dy, wt, dx, g)
        outs.append(dx)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])  # no atomics, fixed summation order
