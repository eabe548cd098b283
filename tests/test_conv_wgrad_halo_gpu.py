"""Direct 3x3 weight-gradient on resident halo / dy tiles (csrc/kernels/conv_wgrad_halo.hip,
tiles 140-142) against fp32 torch: both patch widths, ragged maps (partial patches and row
bands), a pre-padded input (pad 0 geometry on an (H+2) x (W+2) map, as the prepadding conv
layers pass it), a dy channel slice (pixel stride > Cout), several channel pairs and splits.
Each case asserts that the forced tile really ran (gemm.LAST_GLDS)."""
import pytest
import torch

from cxxnet_amd import ops
from cxxnet_amd.ops import gemm
from cxxnet_amd.ops.gemm import ConvGeom

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (N, H, W, C, Cout, tile)
CASES = [
    (2, 56, 56, 64, 64, 140),    # VGG conv1_2-like, width 32 patches
    (2, 28, 28, 128, 64, 140),   # 2 input blocks
    (3, 14, 14, 64, 128, 140),   # 14-wide map: the 16-wide patches win
    (1, 13, 13, 256, 128, 141),  # AlexNet-like 13 x 13, 8 channel pairs
    (2, 20, 37, 64, 64, 141),    # ragged in both directions
    (2, 20, 37, 64, 64, 142),
]


def _rnd(shape, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(*shape, generator=g, device=DEV).to(torch.bfloat16)


def _ref(x, dy, pad):
    C, Cout = x.shape[3], dy.shape[3]
    return torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (Cout, C, 3, 3), dy.float().permute(0, 3, 1, 2),
                                       stride=1, padding=pad)


def _run(x, dy, g, tile):
    Cout, C = g.Cout, g.C
    dw = torch.full((Cout, 3, 3, C), 0.5, device=DEV)
    gemm.set_glds(tile=tile)
    gemm.LAST_GLDS[0] = None
    try:
        ops.conv_backward_weight(x, dy, dw, g)
    finally:
        gemm.set_glds(tile=-1)
    torch.cuda.synchronize()
    assert gemm.LAST_GLDS[0] == tile
    return (dw - 0.5).permute(0, 3, 1, 2)


def _err(got, ref):
    return ((got - ref).norm() / ref.norm()).item()


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_wgrad_halo(case):
    N, H, W, C, Cout, tile = case
    g = ConvGeom(N, H, W, C, H, W, Cout, 3, 3, 1, 1, 1, 1)
    x = _rnd((N, H, W, C), 1)
    dy = _rnd((N, H, W, Cout), 2)
    err = _err(_run(x, dy, g, tile), _ref(x, dy, 1))
    assert err < 1e-2, err


def test_wgrad_halo_prepadded_and_dy_slice():
    N, H, W, C, Cout = 2, 30, 33, 64, 64
    x = _rnd((N, H, W, C), 3)
    xp = torch.zeros(N, H + 2, W + 2, C, device=DEV, dtype=torch.bfloat16)
    xp[:, 1:-1, 1:-1] = x
    big = _rnd((N, H, W, Cout + 64), 4)
    dy = big[..., 32:32 + Cout]  # pixel stride Cout + 64
    g = ConvGeom(N, H + 2, W + 2, C, H, W, Cout, 3, 3, 1, 0, 0, 1)
    err = _err(_run(xp, dy, g, 140), _ref(x, dy.contiguous(), 1))
    assert err < 1e-2, err


def test_wgrad_halo_rejects_unsupported():
    """48 input channels: not a multiple of 64 -- the tile declines and the caller falls back."""
    N, H, W, C, Cout = 1, 12, 12, 48, 64
    g = ConvGeom(N, H, W, C, H, W, Cout, 3, 3, 1, 1, 1, 1)
    x = _rnd((N, H, W, C), 5)
    dy = _rnd((N, H, W, Cout), 6)
    dw = torch.zeros(Cout, 3, 3, C, device=DEV)
    gemm.set_glds(tile=140)
    gemm.LAST_GLDS[0] = None
    try:
        ops.conv_backward_weight(x, dy, dw, g)
    finally:
        gemm.set_glds(tile=-1)
    assert gemm.LAST_GLDS[0] != 140
    err = _err(dw.permute(0, 3, 1, 2), _ref(x, dy, 1))
    assert err < 1e-2, err
