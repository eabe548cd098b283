"""The one-wave-per-SIMD address-free GEMM tile (csrc/kernels/gemm_4w.hip, id 114; the other
4w tiles were retired in round 5) against fp32 torch on the ops that route to it: conv forward
(implicit-im2col gather, padding taps, groups, stride 2, 1x1) and the stride-1 conv
data-gradient; fc forward declines it (K-direct operands are not compiled) and falls back.  Each case asserts that the forced tile really ran (gemm.LAST_GLDS): a tile that
returns "unsupported" would otherwise pass on a fallback kernel."""
import pytest
import torch
import torch.nn.functional as F

from cxxnet_amd import ops
from cxxnet_amd.ops import gemm
from cxxnet_amd.ops.gemm import ConvGeom, conv_out_size

pytestmark = pytest.mark.gpu
DEV = "cuda"
TILES = (114,)


def _rnd(shape, scale, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV) * scale).to(torch.bfloat16)


def _rel(a, ref):
    a, ref = a.float(), ref.float()
    return ((a - ref).norm() / ref.norm().clamp_min(1e-30)).item()


def _geom(N, H, W, C, Cout, K, s, p, G):
    Ho, Wo = conv_out_size(H, W, K, K, s, p, p)
    return ConvGeom(N, H, W, C, Ho, Wo, Cout, K, K, s, p, p, G)


CONV = [
    (8, 14, 14, 128, 256, 3, 1, 1, 1),   # 3x3 pad 1: 18 K-tiles, padding taps at the borders
    (4, 13, 13, 64, 192, 3, 1, 1, 1),    # 9 K-tiles (odd: the peeled last tile), 676 rows
    (4, 12, 12, 256, 256, 3, 1, 1, 2),   # 2 groups of 128 channels
    (4, 15, 15, 64, 128, 3, 2, 1, 1),    # stride 2
    (8, 7, 7, 192, 64, 1, 1, 0, 1),      # 1x1
    (2, 9, 9, 128, 128, 5, 1, 2, 1),     # 5x5 pad 2: 25 taps
]


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("case", CONV, ids=lambda c: "x".join(map(str, c)))
def test_conv_forward(tile, case):
    g = _geom(*case)
    x = _rnd((g.N, g.H, g.W, g.C), 1.0, 1)
    w = _rnd((g.Cout, g.KH, g.KW, g.cg_in), 0.05, 2)
    b = torch.randn(g.Cout, device=DEV) * 0.1
    y = torch.empty(g.N, g.Ho, g.Wo, g.Cout, dtype=torch.bfloat16, device=DEV)
    gemm.set_glds(tile=tile)
    gemm.LAST_GLDS[0] = None
    try:
        ops.conv_forward(x, w, b, y, g, relu=True)
    finally:
        gemm.set_glds(tile=-1)
    assert gemm.LAST_GLDS[0] == tile
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, stride=g.stride,
                   padding=(g.pad_y, g.pad_x), groups=g.groups).clamp_min(0).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("case", [c for c in CONV if c[6] == 1], ids=lambda c: "x".join(map(str, c)))
def test_conv_data_grad(tile, case):
    g = _geom(*case)
    dy = _rnd((g.N, g.Ho, g.Wo, g.Cout), 1.0, 3)
    w = _rnd((g.Cout, g.KH, g.KW, g.cg_in), 0.05, 4)
    dx = torch.empty(g.N, g.H, g.W, g.C, dtype=torch.bfloat16, device=DEV)
    gemm.set_glds(tile=tile)
    gemm.LAST_GLDS[0] = None
    try:
        ops.conv_backward_data(dy, w, dx, g)
    finally:
        gemm.set_glds(tile=-1)
    assert gemm.LAST_GLDS[0] == tile
    ref = torch.nn.grad.conv2d_input((g.N, g.C, g.H, g.W), w.float().permute(0, 3, 1, 2),
                                     dy.float().permute(0, 3, 1, 2), stride=g.stride,
                                     padding=(g.pad_y, g.pad_x), groups=g.groups).permute(0, 2, 3, 1)
    assert _rel(dx, ref) < 1e-2


@pytest.mark.parametrize("nin,nout,B", [(4096, 1000, 96), (1024, 1024, 1024)])
def test_fc_forward_declines(nin, nout, B):
    x = _rnd((B, nin), 1.0, 7)
    w = _rnd((nout, nin), 0.02, 8)
    b = torch.randn(nout, device=DEV) * 0.1
    y = torch.empty(B, nout, dtype=torch.bfloat16, device=DEV)
    gemm.set_glds(tile=114)
    gemm.LAST_GLDS[0] = None
    try:
        ops.fc_forward(x, w, b, y)
    finally:
        gemm.set_glds(tile=-1)
    assert gemm.LAST_GLDS[0] != 114
    assert _rel(y, x.float() @ w.float().t() + b) < 1e-2


def test_unsupported_shapes_fall_back():
    """kdim not a multiple of 64, or a gather with Cg % 64 != 0: the tile declines (-1) and the
    op still computes the right answer on another kernel."""
    g = _geom(4, 13, 13, 48, 128, 3, 1, 1, 1)  # Cg 48
    x = _rnd((g.N, g.H, g.W, g.C), 1.0, 5)
    w = _rnd((g.Cout, g.KH, g.KW, g.cg_in), 0.05, 6)
    y = torch.empty(g.N, g.Ho, g.Wo, g.Cout, dtype=torch.bfloat16, device=DEV)
    gemm.set_glds(tile=114)
    gemm.LAST_GLDS[0] = None
    try:
        ops.conv_forward(x, w, None, y, g)
    finally:
        gemm.set_glds(tile=-1)
    assert gemm.LAST_GLDS[0] != 114
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, padding=1).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 1e-2
