"""The one-wave-per-SIMD MN-major GEMM (csrc/kernels/gemm_4w_mn.hip, tile 120) on the conv
weight-gradient it serves -- implicit-im2col gather of x (padding taps, stride 2, groups,
1x1, channels per group not a multiple of 64), dy direct, fp32 atomic split-K epilogue --
against fp32 torch.  Each case asserts that the forced tile really ran (gemm.LAST_GLDS)."""
import pytest
import torch

from cxxnet_amd import ops
from cxxnet_amd.ops import gemm
from cxxnet_amd.ops.gemm import ConvGeom, conv_out_size

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [
    (8, 13, 13, 256, 384, 3, 1, 1, 1),   # AlexNet conv3 (b8): 2304 columns, 1352 pixels (K tail)
    (4, 13, 13, 384, 256, 3, 1, 1, 2),   # groups of 192 channels: a tile's columns cross taps
    (4, 27, 27, 96, 256, 5, 1, 2, 2),    # AlexNet conv2: 48 channels per group, 25 taps
    (4, 15, 15, 64, 96, 3, 2, 1, 1),     # stride 2, 96 outputs (a partial 128 tile)
    (8, 7, 7, 192, 64, 1, 1, 0, 1),      # 1x1, 49-pixel images (several images per K-tile)
    (2, 56, 56, 64, 64, 3, 1, 1, 1),     # VGG-like: 6272 pixels
]


def _rnd(shape, scale, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c)))
def test_conv_weight_grad(case):
    N, H, W, C, Cout, K, s, p, G = case
    Ho, Wo = conv_out_size(H, W, K, K, s, p, p)
    g = ConvGeom(N, H, W, C, Ho, Wo, Cout, K, K, s, p, p, G)
    x = _rnd((N, H, W, C), 1.0, 1)
    dy = _rnd((N, Ho, Wo, Cout), 1.0, 2)
    dw = torch.full((Cout, K, K, C // G), 0.5, device=DEV)
    gemm.set_glds(tile=120)
    gemm.LAST_GLDS[0] = None
    try:
        ops.conv_backward_weight(x, dy, dw, g)
    finally:
        gemm.set_glds(tile=-1)
    assert gemm.LAST_GLDS[0] == 120
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (Cout, C // G, K, K),
                                      dy.float().permute(0, 3, 1, 2), stride=s, padding=p, groups=G)
    got = (dw - 0.5).permute(0, 3, 1, 2)
    err = ((got - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err
