"""The direct 3x3 halo convolution (csrc/kernels/conv_halo.hip, tile ids 130-131) against fp32
torch: forward (bias + relu epilogue) and the stride-1 data-gradient (plain and relu'-masked),
one and several 64-channel blocks (single and double-buffered halo), 32- and 16-pixel-wide
patches, patches cut by the map's right and bottom edges, output channels not a multiple of the
block.  Each case asserts that the forced tile really ran (gemm.LAST_GLDS)."""
import pytest
import torch
import torch.nn.functional as F

from cxxnet_amd import ops
from cxxnet_amd.ops import gemm
from cxxnet_amd.ops.gemm import ConvGeom

pytestmark = pytest.mark.gpu
DEV = "cuda"
TILES = (130, 131)


def _rnd(shape, scale, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV) * scale).to(torch.bfloat16)


def _rel(a, ref):
    a, ref = a.float(), ref.float()
    return ((a - ref).norm() / ref.norm().clamp_min(1e-30)).item()


CASES = [
    (2, 16, 64, 64, 64),      # W % 32 == 0: 32-wide patches, one channel block
    (2, 20, 48, 128, 128),    # 16-wide patches (48 % 32 != 0), two blocks, bottom edge cut
    (1, 9, 40, 192, 64),      # three blocks: the halo buffers alternate 0 1 0
    (3, 8, 36, 64, 136),      # right edge cut (36 = 2 x 16 + 4), 136 outputs: a partial block
    (1, 24, 112, 128, 128),   # VGG conv2_2's width
]


def _geom(N, H, W, C, Cout):
    return ConvGeom(N, H, W, C, H, W, Cout, 3, 3, 1, 1, 1, 1)


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_halo_forward(tile, case):
    g = _geom(*case)
    x = _rnd((g.N, g.H, g.W, g.C), 1.0, 1)
    w = _rnd((g.Cout, 3, 3, g.C), 0.05, 2)
    b = torch.randn(g.Cout, device=DEV) * 0.1
    y = torch.full((g.N, g.H, g.W, g.Cout), 9.0, dtype=torch.bfloat16, device=DEV)
    gemm.set_glds(tile=tile)
    gemm.LAST_GLDS[0] = None
    try:
        ops.conv_forward(x, w, b, y, g, relu=True)
    finally:
        gemm.set_glds(tile=-1)
    assert gemm.LAST_GLDS[0] == tile
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=1)
    assert _rel(y, ref.clamp_min(0).permute(0, 2, 3, 1)) < 1e-2


# (the data-gradient gathers dy: its Cout is the blocked channel count, C the output rows)
DGRAD = [(2, 16, 64, 64, 64), (2, 20, 48, 128, 128), (1, 9, 40, 64, 192), (3, 8, 36, 72, 128)]


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("mask", [False, True])
@pytest.mark.parametrize("case", DGRAD, ids=lambda c: "x".join(map(str, c)))
def test_halo_data_grad(tile, mask, case):
    g = _geom(*case)
    dy = _rnd((g.N, g.H, g.W, g.Cout), 1.0, 3)
    w = _rnd((g.Cout, 3, 3, g.C), 0.05, 4)
    z = _rnd((g.N, g.H, g.W, g.C), 1.0, 5)  # relu(z) in dx on entry when masked
    dx = z.clamp_min(0) if mask else torch.empty_like(z)
    gemm.set_glds(tile=tile)
    gemm.LAST_GLDS[0] = None
    try:
        ops.conv_backward_data(dy, w, dx, g, mask_relu=mask)
    finally:
        gemm.set_glds(tile=-1)
    assert gemm.LAST_GLDS[0] == tile
    ref = torch.nn.grad.conv2d_input((g.N, g.C, g.H, g.W), w.float().permute(0, 3, 1, 2),
                                     dy.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    if mask:
        ref = ref * (z.float() > 0)
    assert _rel(dx, ref) < 1e-2


def test_halo_declines_other_convs():
    """Stride 2, 5x5 or channel blocks that are not whole: the tile declines (-1) and the op
    still computes the right answer on another kernel."""
    for geo in (ConvGeom(2, 16, 16, 64, 8, 8, 64, 3, 3, 2, 1, 1, 1), ConvGeom(2, 16, 16, 48, 16, 16, 64, 3, 3, 1, 1, 1, 1)):
        x = _rnd((geo.N, geo.H, geo.W, geo.C), 1.0, 6)
        w = _rnd((geo.Cout, 3, 3, geo.C), 0.05, 7)
        y = torch.empty(geo.N, geo.Ho, geo.Wo, geo.Cout, dtype=torch.bfloat16, device=DEV)
        gemm.set_glds(tile=130)
        gemm.LAST_GLDS[0] = None
        try:
            ops.conv_forward(x, w, None, y, geo)
        finally:
            gemm.set_glds(tile=-1)
        assert gemm.LAST_GLDS[0] != 130
        ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, stride=geo.stride, padding=1)
        assert _rel(y, ref.permute(0, 2, 3, 1)) < 1e-2


# persistent forms (one output-channel block; any number of 64-channel input blocks):
# (N, H, W, C, Cout)
PS_TILES = {133: 128}
PS_CASES = [
    (2, 16, 64, 64, 64),     # two 32-wide x 8-row patches per row band, whole patches
    (3, 20, 48, 64, 64),     # 16-wide patches, bottom edge cut
    (1, 9, 36, 64, 40),      # right edge cut, 40 of 64 output channels
    (24, 16, 32, 64, 64),    # 48 patches: several per block on every XCD share
    (2, 24, 112, 64, 128),   # VGG conv2_1's width (16-wide patches)
    (5, 16, 64, 128, 128),   # two channel blocks per patch (conv2_2)
    (3, 12, 40, 192, 64),    # three channel blocks, cut edges
]


@pytest.mark.parametrize("tile", sorted(PS_TILES))
@pytest.mark.parametrize("case", PS_CASES, ids=lambda c: "x".join(map(str, c)))
def test_halo_persistent_forward(tile, case):
    N, H, W, C, Cout = case
    if Cout > PS_TILES[tile]:
        pytest.skip("more output channels than the persistent block")
    g = _geom(N, H, W, C, Cout)
    x = _rnd((N, H, W, C), 1.0, 11)
    w = _rnd((Cout, 3, 3, C), 0.05, 12)
    b = torch.randn(Cout, device=DEV) * 0.1
    y = torch.full((N, H, W, Cout), 9.0, dtype=torch.bfloat16, device=DEV)
    gemm.set_glds(tile=tile)
    gemm.LAST_GLDS[0] = None
    try:
        ops.conv_forward(x, w, b, y, g, relu=True)
    finally:
        gemm.set_glds(tile=-1)
    assert gemm.LAST_GLDS[0] == tile
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=1)
    assert _rel(y, ref.clamp_min(0).permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("tile", sorted(PS_TILES))
@pytest.mark.parametrize("mask", [False, True])
@pytest.mark.parametrize("cin", [64, 128])
def test_halo_persistent_data_grad(tile, mask, cin):
    N, H, W = 6, 24, 64  # dy cin channels (the blocked operand) -> dx 64 channels
    g = _geom(N, H, W, 64, cin)
    dy = _rnd((N, H, W, cin), 1.0, 13)
    w = _rnd((cin, 3, 3, 64), 0.05, 14)
    z = _rnd((N, H, W, 64), 1.0, 15)
    dx = z.clamp_min(0) if mask else torch.empty_like(z)
    gemm.set_glds(tile=tile)
    gemm.LAST_GLDS[0] = None
    try:
        ops.conv_backward_data(dy, w, dx, g, mask_relu=mask)
    finally:
        gemm.set_glds(tile=-1)
    assert gemm.LAST_GLDS[0] == tile
    ref = torch.nn.grad.conv2d_input((N, 64, H, W), w.float().permute(0, 3, 1, 2),
                                     dy.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    if mask:
        ref = ref * (z.float() > 0)
    assert _rel(dx, ref) < 1e-2


def test_halo_persistent_declines_two_output_blocks():
    """256 output channels on the 128-channel persistent block: 133 declines."""
    geo = _geom(2, 16, 32, 64, 256)
    x = _rnd((2, 16, 32, 64), 1.0, 16)
    w = _rnd((256, 3, 3, 64), 0.05, 17)
    y = torch.empty(2, 16, 32, 256, dtype=torch.bfloat16, device=DEV)
    gemm.set_glds(tile=133)
    gemm.LAST_GLDS[0] = None
    try:
        ops.conv_forward(x, w, None, y, geo)
    finally:
        gemm.set_glds(tile=-1)
    assert gemm.LAST_GLDS[0] != 133
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, padding=1)
    assert _rel(y, ref.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("mask", [False, True])
@pytest.mark.parametrize("case", [(2, 16, 64, 64, 64), (3, 20, 48, 128, 128), (2, 9, 40, 64, 192), (1, 13, 13, 128, 256)],
                         ids=lambda c: "x".join(map(str, c)))
def test_halo_data_grad_bias_sum(tile, mask, case):
    """EPI_BF16_DB on the halo tiles: dx exactly as the plain epilogue writes it, and dbias += the
    column sums of the stored (relu'-masked) dx, from per-(patch, wave) partial rows."""
    g = _geom(*case)
    dy = _rnd((g.N, g.H, g.W, g.Cout), 1.0, 21)
    w = _rnd((g.Cout, 3, 3, g.C), 0.05, 22)
    z = _rnd((g.N, g.H, g.W, g.C), 1.0, 23)
    gemm.set_glds(tile=tile)
    try:
        dx_ref = z.clamp_min(0) if mask else torch.empty_like(z)
        ops.conv_backward_data(dy, w, dx_ref, g, mask_relu=mask)
        dx = z.clamp_min(0) if mask else torch.empty_like(z)
        db = torch.full((g.C,), 0.25, device=DEV)
        gemm.LAST_GLDS[0] = None
        fused = ops.conv_backward_data(dy, w, dx, g, mask_relu=mask, dbias=db)
    finally:
        gemm.set_glds(tile=-1)
    torch.cuda.synchronize()
    assert fused and gemm.LAST_GLDS[0] == tile
    assert torch.equal(dx, dx_ref)
    ref = 0.25 + dx_ref.float().reshape(-1, g.C).sum(0)
    assert _rel(db, ref) < 1e-3
