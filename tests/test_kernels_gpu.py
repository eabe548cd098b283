"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op.

Inputs are rounded to bf16 first; the reference then runs in fp32 on the CPU on
those exact values, so the only differences are bf16 output rounding and fp32
summation order.  (This is the pairtest idea of reference
src/layer/pairtest_layer-inl.hpp, with torch as the slave implementation.)
"""
import pytest
import torch

from cxxnet_amd import ops
from cxxnet_amd.ops.gemm import ConvGeom, conv_out_size

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).float()


def relerr(a, b):
    a = a.float().cpu()
    b = b.float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


CONV_CASES = [
    # N, C(phys), H, W, Cout, K, stride, pad, groups
    (2, 4, 227, 227, 96, 11, 4, 0, 1),     # AlexNet conv1 (3 channels padded to 4)
    (2, 96, 27, 27, 256, 5, 1, 2, 2),      # AlexNet conv2 (grouped)
    (3, 256, 13, 13, 384, 3, 1, 1, 1),     # AlexNet conv3
    (2, 384, 13, 13, 256, 3, 1, 1, 2),     # AlexNet conv5
    (2, 64, 17, 19, 40, 1, 1, 0, 1),       # 1x1, ragged spatial / Cout
    (2, 32, 15, 15, 48, 3, 2, 1, 1),       # strided 3x3 (strided dgrad path)
    (1, 8, 9, 9, 16, 5, 1, 2, 1),
]


def _geom(N, C, H, W, Cout, K, s, p, g):
    Ho, Wo = conv_out_size(H, W, K, K, s, p, p)
    return ConvGeom(N, H, W, C, Ho, Wo, Cout, K, K, s, p, p, g)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_forward(case):
    geo = _geom(*case)
    x = rnd(geo.N, geo.H, geo.W, geo.C, seed=1)
    w = rnd(geo.Cout, geo.KH, geo.KW, geo.cg_in, scale=0.05, seed=2)
    b = rnd(geo.Cout, scale=0.1, seed=3)
    y_ref = torch.empty(geo.N, geo.Ho, geo.Wo, geo.Cout)
    ops.conv_forward(x, w, b, y_ref, geo, relu=True)
    y = torch.empty(geo.N, geo.Ho, geo.Wo, geo.Cout, dtype=torch.bfloat16, device=DEV)
    ops.conv_forward(x.to(DEV, torch.bfloat16), w.to(DEV, torch.bfloat16), b.to(DEV), y, geo, relu=True)
    torch.cuda.synchronize()
    assert relerr(y, y_ref) < 2e-2


@pytest.mark.parametrize("case", CONV_CASES[1:])
def test_conv_backward_data(case):
    geo = _geom(*case)
    dy = rnd(geo.N, geo.Ho, geo.Wo, geo.Cout, seed=4)
    w = rnd(geo.Cout, geo.KH, geo.KW, geo.cg_in, scale=0.05, seed=5)
    dx_ref = torch.empty(geo.N, geo.H, geo.W, geo.C)
    ops.conv_backward_data(dy, w, dx_ref, geo)
    dx = torch.empty(geo.N, geo.H, geo.W, geo.C, dtype=torch.bfloat16, device=DEV)
    ops.conv_backward_data(dy.to(DEV, torch.bfloat16), w.to(DEV, torch.bfloat16), dx, geo)
    torch.cuda.synchronize()
    assert relerr(dx, dx_ref) < 2e-2


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_backward_weight(case):
    geo = _geom(*case)
    x = rnd(geo.N, geo.H, geo.W, geo.C, seed=6)
    dy = rnd(geo.N, geo.Ho, geo.Wo, geo.Cout, seed=7)
    init = rnd(geo.Cout, geo.KH, geo.KW, geo.cg_in, seed=8)
    dw_ref = init.clone()
    ops.conv_backward_weight(x, dy, dw_ref, geo)
    dw = init.to(DEV).clone()
    ops.conv_backward_weight(x.to(DEV, torch.bfloat16), dy.to(DEV, torch.bfloat16), dw, geo)
    torch.cuda.synchronize()
    assert relerr(dw, dw_ref) < 1e-2


FC_CASES = [(256, 9216, 4096), (100, 784, 100), (100, 100, 10), (64, 256, 121), (32, 4096, 1000)]


@pytest.mark.parametrize("B,nin,nout", FC_CASES)
def test_fc(B, nin, nout):
    x = rnd(B, nin, seed=9)
    w = rnd(nout, nin, scale=0.02, seed=10)
    b = rnd(nout, scale=0.1, seed=11)
    dy = rnd(B, nout, seed=12)
    y_ref = torch.empty(B, nout)
    ops.fc_forward(x, w, b, y_ref)
    dx_ref = torch.empty(B, nin)
    ops.fc_backward_data(dy, w, dx_ref)
    dw_ref = torch.ones(nout, nin)
    ops.fc_backward_weight(x, dy, dw_ref)

    xd, wd, dyd = (t.to(DEV, torch.bfloat16) for t in (x, w, dy))
    y = torch.empty(B, nout, dtype=torch.bfloat16, device=DEV)
    ops.fc_forward(xd, wd, b.to(DEV), y)
    dx = torch.empty(B, nin, dtype=torch.bfloat16, device=DEV)
    ops.fc_backward_data(dyd, wd, dx)
    dw = torch.ones(nout, nin, device=DEV)
    ops.fc_backward_weight(xd, dyd, dw)
    torch.cuda.synchronize()
    assert relerr(y, y_ref) < 2e-2
    assert relerr(dx, dx_ref) < 2e-2
    assert relerr(dw, dw_ref) < 1e-2
    # fused relu: forward with relu epilogue, data-grad masked by the stored activation
    y_ref.copy_(torch.clamp_min(x @ w.t() + b, 0))
    ops.fc_forward(xd, wd, b.to(DEV), y, relu=True)
    assert relerr(y, y_ref) < 2e-2
    act = rnd(B, nin, seed=15).clamp_min(0)
    dxm_ref = act.clone()
    ops.fc_backward_data(dy, w, dxm_ref, mask_relu=True)
    dxm = act.to(DEV, torch.bfloat16)
    ops.fc_backward_data(dyd, wd, dxm, mask_relu=True)
    torch.cuda.synchronize()
    assert relerr(dxm, dxm_ref) < 2e-2


@pytest.mark.parametrize("mode,relu,k,s,p,C", [("max", False, 3, 2, 0, 96), ("max", True, 3, 2, 0, 256),
                                               ("avg", False, 3, 1, 1, 64), ("sum", False, 2, 2, 0, 8),
                                               ("max", False, 3, 2, 0, 3)])
def test_pool(mode, relu, k, s, p, C):
    N, H, W = 2, 27, 27
    Ho = ops.pool_out_size(H, k, s, p)
    x = rnd(N, H, W, C, seed=13)
    dy = rnd(N, Ho, Ho, C, seed=14)
    y_ref = torch.empty(N, Ho, Ho, C)
    st_ref = torch.empty(N, Ho, Ho, C, dtype=torch.uint8)
    ops.pool_forward(x, y_ref, st_ref, k, k, s, p, mode, relu)
    dx_ref = torch.empty_like(x)
    ops.pool_backward(x, st_ref, dy, dx_ref, k, k, s, p, mode, relu)

    xd = x.to(DEV, torch.bfloat16)
    y = torch.empty(N, Ho, Ho, C, dtype=torch.bfloat16, device=DEV)
    st = torch.empty(N, Ho, Ho, C, dtype=torch.uint8, device=DEV)
    ops.pool_forward(xd, y, st, k, k, s, p, mode, relu)
    dx = torch.empty_like(xd)
    ops.pool_backward(xd, st, dy.to(DEV, torch.bfloat16), dx, k, k, s, p, mode, relu)
    torch.cuda.synchronize()
    assert relerr(y, y_ref) < 1e-2
    if mode == "max":
        # inputs are exact bf16 values, so the first-max positions must agree exactly
        assert torch.equal(st.cpu(), st_ref)
    assert relerr(dx, dx_ref) < 2e-2


@pytest.mark.parametrize("relu_fwd", [False, True])
def test_pool_mask_in_state(relu_fwd):
    """Max pool over relu'd (or relu-in-pool) input: relu' encoded in the offsets
    (bit 7) gives the same gradient as reading x."""
    N, H, W, C, k, s = 2, 27, 27, 96, 3, 2
    Ho = ops.pool_out_size(H, k, s, 0)
    x = rnd(N, H, W, C, seed=21)
    if not relu_fwd:
        x = x.clamp_min(0)  # fused conv->relu producer
    dy = rnd(N, Ho, Ho, C, seed=22)
    y_ref = torch.empty(N, Ho, Ho, C)
    st_ref = torch.empty(N, Ho, Ho, C, dtype=torch.uint8)
    ops.pool_forward(x, y_ref, st_ref, k, k, s, 0, "max", relu_fwd)
    dx_ref = torch.empty_like(x)
    ops.pool_backward(x, st_ref, dy, dx_ref, k, k, s, 0, "max", True)
    xd = x.to(DEV, torch.bfloat16)
    y = torch.empty(N, Ho, Ho, C, dtype=torch.bfloat16, device=DEV)
    st = torch.empty(N, Ho, Ho, C, dtype=torch.uint8, device=DEV)
    ops.pool_forward(xd, y, st, k, k, s, 0, "max", relu_fwd, mark_mask=True)
    assert (st.cpu() >= 0x80).any()  # some windows are all <= 0
    dx = torch.empty_like(xd)
    db = torch.full((C,), 0.5, device=DEV)
    ops.pool_backward(xd, st, dy.to(DEV, torch.bfloat16), dx, k, k, s, 0, "max", 2, dbias=db)
    torch.cuda.synchronize()
    assert relerr(dx, dx_ref) < 2e-2
    # folded bias gradient of the producing conv: 0.5 + column sums of dx
    assert relerr(db, 0.5 + dx_ref.reshape(-1, C).sum(0)) < 2e-2


@pytest.mark.parametrize("mask", [False, True])
@pytest.mark.parametrize("C,nsize", [(96, 5), (256, 5), (40, 3), (64, 9), (1024, 5)])
def test_lrn(C, nsize, mask):
    """Shuffle kernels (C <= 512: whole pixels per wave, halo by ds_bpermute; odd pixel
    count leaves a partial last wave) and the LDS fallback (C = 1024).  mask: the input is
    relu(z) of a fused producer (about half the values exactly 0) and the data-gradient is
    also multiplied by relu'(z)."""
    N, H, W = 2, 13, 13
    x = rnd(N, H, W, C, scale=2.0, seed=15)
    if mask:
        x = x.clamp_min(0)
    dy = rnd(N, H, W, C, seed=16)
    args = (nsize, 0.001, 0.75, 1.0)
    y_ref = torch.empty_like(x)
    ops.lrn_forward(x, y_ref, *args)
    dx_ref = torch.empty_like(x)
    ops.lrn_backward(x, dy, dx_ref, *args, mask_relu=mask)
    if mask:
        assert (dx_ref[x == 0] == 0).all() and (dx_ref[x > 0] != 0).any()
    xd = x.to(DEV, torch.bfloat16)
    y = torch.empty_like(xd)
    ops.lrn_forward(xd, y, *args)
    dx = torch.empty_like(xd)
    ops.lrn_backward(xd, dy.to(DEV, torch.bfloat16), dx, *args, mask_relu=mask)
    xi = xd.clone()
    ops.lrn_backward(xi, dy.to(DEV, torch.bfloat16), xi, *args, mask_relu=mask)  # in place (the layer's usage)
    torch.cuda.synchronize()
    assert relerr(y, y_ref) < 1e-2
    assert relerr(dx, dx_ref) < 2e-2
    assert torch.equal(xi, dx)


@pytest.mark.parametrize("C,nsize,mask,npix", [(192, 5, True, 2 * 56 * 56), (64, 5, False, 3 * 13 * 13),
                                                (256, 3, True, 2 * 7 * 7), (512, 9, True, 1000)])
def test_lrn_backward_bias(C, nsize, mask, npix):
    """LRN backward with the conv-in-front's bias gradient summed on the way out
    (ops.lrn_backward_bias, GoogLeNet norm2): dx as the plain kernel's (in place bitwise as out
    of place), db += the column sums of the stored bf16 dx against an fp32 sum; pixel counts that leave
    partial waves, more groups than blocks (grid-stride) and C / 8 not dividing 64."""
    xd = rnd(1, 1, npix, C, scale=2.0, seed=21).to(DEV, torch.bfloat16)
    if mask:
        xd = xd.clamp_min(0)
    dy = rnd(1, 1, npix, C, seed=22).to(DEV, torch.bfloat16)
    args = (nsize, 0.001, 0.75, 1.0)
    dx_ref = torch.empty_like(xd)
    ops.lrn_backward(xd, dy, dx_ref, *args, mask_relu=mask)
    db = torch.full((C,), 0.5, device=DEV)
    dx = torch.empty_like(xd)
    assert ops.lrn_backward_bias(xd, dy, dx, *args, db, mask_relu=mask)
    xi = xd.clone()
    db2 = torch.full((C,), 0.5, device=DEV)
    assert ops.lrn_backward_bias(xi, dy, xi, *args, db2, mask_relu=mask)
    torch.cuda.synchronize()
    assert torch.equal(xi, dx)  # in place: the same values
    assert relerr(dx, dx_ref) < 1e-2  # (the two kernels may contract the arithmetic differently)
    ref = dx.float().reshape(-1, C).sum(0)
    assert relerr(db - 0.5, ref) < 1e-5
    assert relerr(db2 - 0.5, ref) < 1e-5


@pytest.mark.parametrize("kind", ["relu", "sigmoid", "tanh", "xelu"])
def test_activation(kind):
    x = rnd(1003, seed=17)
    dy = rnd(1003, seed=18)
    y_ref = torch.empty_like(x)
    ops.act_forward(kind, x, y_ref)
    y_ref_b = y_ref.to(torch.bfloat16).float()
    dx_ref = torch.empty_like(x)
    ops.act_backward(kind, y_ref_b, dy, dx_ref)
    xd = x.to(DEV, torch.bfloat16)
    y = torch.empty_like(xd)
    y2 = torch.empty_like(xd)
    ops.act_forward(kind, xd, y, y2)
    dx = torch.empty_like(xd)
    ops.act_backward(kind, y, dy.to(DEV, torch.bfloat16), dx)
    torch.cuda.synchronize()
    assert relerr(y, y_ref) < 1e-2 and torch.equal(y, y2)
    assert relerr(dx, dx_ref) < 1e-2


def test_dropout_mask_matches_reference():
    n = 4099
    x = rnd(n, seed=19)
    y_ref = torch.empty_like(x)
    ops.dropout_apply(x, y_ref, 1234, 0.5)
    y = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    ops.dropout_apply(x.to(DEV, torch.bfloat16), y, 1234, 0.5)
    torch.cuda.synchronize()
    assert relerr(y, y_ref) < 1e-2
    keep = (y.cpu() != 0).float().mean().item()
    assert 0.45 < keep < 0.55


@pytest.mark.parametrize("rows,K", [(37, 1000), (16, 10), (33, 300), (5, 700), (9, 1500)])
def test_softmax_and_loss_grad(rows, K):
    """register-resident rows (K <= 1024: 4 / 8 / 16 values per lane) and the strided kernel"""
    x = rnd(rows, K, scale=3.0, seed=20)
    label = torch.randint(0, K, (rows, 1)).float()
    p_ref = torch.empty_like(x)
    p32_ref = torch.empty_like(x)
    ops.softmax_forward(x, p_ref, p32_ref)
    g_ref = p_ref.clone()
    ops.loss_grad("softmax", g_ref, label, 0.5, p32_ref)
    xd = x.to(DEV, torch.bfloat16)
    p = torch.empty_like(xd)
    p32 = torch.empty(rows, K, device=DEV)
    ops.softmax_forward(xd, p, p32)
    ops.loss_grad("softmax", p, label.to(DEV), 0.5, p32)
    torch.cuda.synchronize()
    assert relerr(p32, p32_ref) < 1e-2
    assert relerr(p, g_ref) < 1e-2


@pytest.mark.parametrize("rows,C", [(30000, 96), (256, 4096), (100, 10)])
def test_bias_grad(rows, C):
    dy = rnd(rows, C, seed=21)
    db_ref = torch.ones(C)
    ops.bias_grad(dy, db_ref)
    db = torch.ones(C, device=DEV)
    ops.bias_grad(dy.to(DEV, torch.bfloat16), db)
    torch.cuda.synchronize()
    assert relerr(db, db_ref) < 1e-3


@pytest.mark.parametrize("n", [10007, 4200011])  # the large case runs the 2-deep unrolled loop
@pytest.mark.parametrize("algo", ["sgd", "nag", "adam"])
def test_fused_update(algo, n):
    w = rnd(n, seed=22)
    g = rnd(n, seed=23)
    m = rnd(n, scale=0.1, seed=24)
    m2 = rnd(n, scale=0.1, seed=25).abs()
    # 4-aligned segments with and without a < 4 tail, and an unaligned slice (element-wise path)
    a = n // 2 // 4 * 4
    segs = [(0, a, 0.01, 0.0005, 0.9, 0.0), (a, 3001, 0.02, 0.0, 0.9, 0.5),
            (a + 3001, n - a - 3001, 0.03, 0.001, 0.8, 0.0)]
    ref = [t.clone() for t in (w, g, m, m2)]
    wb_ref = torch.empty(n)
    ops.fused_update(algo, ref[0], ref[1], ref[2], ref[3], wb_ref, segs)
    dev = [t.to(DEV) for t in (w, g, m, m2)]
    wb = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    ops.fused_update(algo, dev[0], dev[1], dev[2], dev[3], wb, segs)
    torch.cuda.synchronize()
    assert relerr(dev[0], ref[0]) < 1e-5
    assert relerr(dev[2], ref[2]) < 1e-5
    if algo == "adam":
        assert relerr(dev[3], ref[3]) < 1e-5
    assert dev[1].abs().max().item() == 0.0
    assert relerr(wb, ref[0]) < 1e-2


def test_layout_roundtrip():
    x = torch.randn(2, 3, 11, 13)
    node = torch.empty(2, 11, 13, 4, dtype=torch.bfloat16, device=DEV)
    ops.input_to_nhwc(x.to(DEV), node)
    back = ops.nhwc_to_nchw(node, 3)
    torch.cuda.synchronize()
    assert relerr(back, x) < 1e-2
    assert node[..., 3].abs().max().item() == 0
    # flatten transpose
    t = rnd(2, 6 * 6, 256, seed=26)
    out = torch.empty(2, 256 * 36, dtype=torch.bfloat16, device=DEV)
    ops.transpose(t.to(DEV, torch.bfloat16), out, 2, 36, 256)
    ref = t.transpose(1, 2).reshape(2, -1)
    torch.cuda.synchronize()
    assert relerr(out, ref) < 1e-2


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_image_u8_to_nhwc(mode):
    """Fused augment arithmetic (mean / contrast / illumination / scale / mirror-aware
    mean lookup) against U8Images.to_float."""
    from cxxnet_amd.io.data import U8Images
    g = torch.Generator().manual_seed(mode)
    B, h, w, C, Cp = 5, 13, 17, 3, 4
    pix = torch.randint(0, 256, (B, h, w, C), generator=g, dtype=torch.uint8)
    prm = torch.zeros((B, 4), dtype=torch.int32)
    prm[:, 0] = torch.randint(0, 4, (B,), generator=g)
    prm[:, 1] = torch.randint(0, 6, (B,), generator=g)
    prm[:, 2] = torch.tensor([0, 1, 0, 1, 1])
    cm = torch.stack([torch.rand(B, generator=g) + 0.5, torch.rand(B, generator=g) * 10 - 5], 1)
    mean = {0: None, 1: torch.tensor([100.0, 110.0, 120.0]),
            2: torch.rand((C, h + 3, w + 5), generator=g) * 255,
            3: torch.rand((C, h, w), generator=g) * 255}[mode]
    img = U8Images(pix, prm, cm, mean, mode, 1.0 / 64)
    ref = img.to_float().permute(0, 2, 3, 1)
    out = torch.empty((B, h, w, Cp), dtype=torch.bfloat16, device=DEV)
    ops.image_to_nhwc(img, out)
    got = out.float().cpu()
    assert relerr(got[..., :C], ref) < 1e-2
    assert got[..., C:].abs().max().item() == 0


@pytest.mark.parametrize("mode", [0, 1])
def test_image_u8_fast_path(mode):
    """C=3 -> Cp=4, 4 pixels per thread (pixel count % 4 == 0), batches straddled by quads."""
    from cxxnet_amd.io.data import U8Images
    g = torch.Generator().manual_seed(7 + mode)
    B, h, w = 4, 9, 7  # 63 pixels per image: quads cross image boundaries
    pix = torch.randint(0, 256, (B, h, w, 3), generator=g, dtype=torch.uint8)
    cm = torch.stack([torch.rand(B, generator=g) + 0.5, torch.rand(B, generator=g) * 10 - 5], 1)
    img = U8Images(pix, torch.zeros((B, 4), dtype=torch.int32), cm, torch.tensor([120.0, 110.0, 100.0]), mode, 0.02)
    ref = img.to_float().permute(0, 2, 3, 1)
    out = torch.empty((B, h, w, 4), dtype=torch.bfloat16, device=DEV)
    ops.image_to_nhwc(img, out)
    got = out.float().cpu()
    assert relerr(got[..., :3], ref) < 1e-2
    assert got[..., 3].abs().max().item() == 0


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("w", [7, 13, 227])
def test_image_u8_row_padded_c3(mode, w):
    """3-channel node with rows padded to a multiple of 4 pixels (the first-conv row-run layout,
    NeuralNet._pad_input_channels): image_u8c3_nhwc3p (modes 0/1) and the generic kernel (mode 2)
    write the logical columns, the pad columns stay zero; input_to_nhwc / nhwc_to_nchw honour the
    pitch too."""
    from cxxnet_amd.io.data import U8Images
    g = torch.Generator().manual_seed(11 * w + mode)
    B, h = 3, 5
    wp = (w + 3) // 4 * 4 + (4 if w == 13 else 0)  # one case with more than the minimal pad
    pix = torch.randint(0, 256, (B, h, w, 3), generator=g, dtype=torch.uint8)
    prm = torch.zeros((B, 4), dtype=torch.int32)
    cm = torch.stack([torch.rand(B, generator=g) + 0.5, torch.rand(B, generator=g) * 10 - 5], 1)
    mean = {0: None, 1: torch.tensor([100.0, 110.0, 120.0]), 2: torch.rand((3, h + 2, w + 3), generator=g) * 255}[mode]
    if mode == 2:
        prm[:, 0], prm[:, 1], prm[:, 2] = 1, 2, torch.tensor([0, 1, 0])
    img = U8Images(pix, prm, cm, mean, mode, 1.0 / 64)
    ref = img.to_float().permute(0, 2, 3, 1)
    out = torch.zeros((B, h, wp, 3), dtype=torch.bfloat16, device=DEV)
    ops.image_to_nhwc(img, out)
    got = out.float().cpu()
    assert relerr(got[:, :, :w], ref) < 1e-2
    assert got[:, :, w:].abs().max().item() == 0
    back = ops.nhwc_to_nchw(out, 3, w)
    x = torch.randn(B, 3, h, w)
    node = torch.zeros((B, h, wp, 3), dtype=torch.bfloat16, device=DEV)
    ops.input_to_nhwc(x.to(DEV), node)
    torch.cuda.synchronize()
    assert relerr(back.cpu(), ref.permute(0, 3, 1, 2)) < 1e-2
    assert relerr(ops.nhwc_to_nchw(node, 3, w).cpu(), x) < 1e-2
    assert node[:, :, w:].abs().max().item() == 0


@pytest.mark.parametrize("N", [2, 16])
def test_conv1_three_channel_row_runs(N):
    """AlexNet conv1 (11x11 / 4, 96 outputs) on the 3-channel row-padded node: forward (K_ROWGATHER,
    K = 11 x 40) and weight-gradient (row-run MN gather) against fp32 torch on the same bf16 values."""
    import torch.nn.functional as F
    from cxxnet_amd.ops import gemm as G
    torch.manual_seed(N)
    H = W = 227
    x3 = torch.randn(N, 3, H, W, device=DEV).to(torch.bfloat16).float()
    w3 = (torch.randn(96, 3, 11, 11, device=DEV) * 0.05).to(torch.bfloat16).float()
    dy = torch.randn(N, 96, 55, 55, device=DEV).to(torch.bfloat16).float()
    y_ref = F.conv2d(x3, w3, stride=4) + 0.5
    dw_ref = torch.nn.grad.conv2d_weight(x3, w3.shape, dy, stride=4)
    x = torch.zeros(N, H, 228, 3, device=DEV, dtype=torch.bfloat16)
    x[:, :, :W] = x3.permute(0, 2, 3, 1).to(torch.bfloat16)
    w = w3.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    g = ConvGeom(N, H, 228, 3, 55, 55, 96, 11, 11, 4, 0, 0, 1)
    assert G.rowrun_ok(g)
    y = torch.empty(N, 55, 55, 96, device=DEV, dtype=torch.bfloat16)
    ops.conv_forward(x, w, torch.full((96,), 0.5, device=DEV), y, g)
    dw = torch.full((96, 11, 11, 3), 0.25, device=DEV)
    ops.conv_backward_weight(x, dy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16), dw, g)
    torch.cuda.synchronize()
    assert relerr(y.permute(0, 3, 1, 2), y_ref) < 1e-2
    assert relerr(dw.permute(0, 3, 1, 2) - 0.25, dw_ref) < 1e-2


@pytest.mark.parametrize("N,H,W,C,Cout,K,S,relu", [(2, 227, 228, 3, 96, 11, 4, True), (3, 227, 228, 3, 96, 11, 4, False),
                                                   (40, 227, 228, 3, 96, 11, 4, True),  # 2-3 work items per block
                                                   (2, 35, 35, 4, 32, 5, 2, True), (2, 43, 44, 3, 128, 7, 4, False),
                                                   (5, 30, 32, 3, 64, 3, 4, True),
                                                   (2, 34, 36, 4, 64, 4, 2, True)])  # even KH: no unpaired row
def test_conv_rowrun_direct_forward(N, H, W, C, Cout, K, S, relu):
    """conv_rowrun.hip (input rows staged once per 4 output rows, LDS-DMA double buffer) called
    directly -- it must serve the shape (rc 0, no GEMM fallback) -- against fp32 torch."""
    import torch.nn.functional as F
    from cxxnet_amd import native
    from cxxnet_amd.ops import gemm as G
    torch.manual_seed(N * 7 + K)
    x = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(Cout, K, K, C, device=DEV) * 0.05).to(torch.bfloat16)
    b = torch.randn(Cout, device=DEV)
    Ho, Wo = (H - K) // S + 1, (W - K) // S + 1
    g = ConvGeom(N, H, W, C, Ho, Wo, Cout, K, K, S, 0, 0, 1)
    wp, lp = G._row_padded_weights(w, g)
    y = torch.full((N, Ho, Wo, Cout), 7.0, device=DEV, dtype=torch.bfloat16)
    rc = native.kernels().cxn_conv_rowrun_fwd(x.data_ptr(), x.numel() * 2, wp.data_ptr(), b.data_ptr(), y.data_ptr(),
                                              N, H, W, C, Ho, Wo, Cout, K, lp, S, Cout, int(relu),
                                              torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, stride=S)
    if relu:
        ref = ref.clamp_min(0)
    assert relerr(y.permute(0, 3, 1, 2), ref) < 1e-2


def test_conv1_three_channel_row_runs_deterministic():
    """Deterministic mode (left on by a trainer with deterministic = 1) keeps the 3-channel
    row-run weight-gradient: one K slice, bitwise equal on a repeat, and still exact."""
    from cxxnet_amd.ops import gemm as G
    G.set_deterministic(True)
    test_conv1_three_channel_row_runs(2)
    torch.manual_seed(5)
    N = 2
    x = torch.zeros(N, 227, 228, 3, device=DEV, dtype=torch.bfloat16)
    x[:, :, :227] = torch.randn(N, 227, 227, 3, device=DEV).to(torch.bfloat16)
    dy = torch.randn(N, 55, 55, 96, device=DEV).to(torch.bfloat16)
    g = ConvGeom(N, 227, 228, 3, 55, 55, 96, 11, 11, 4, 0, 0, 1)
    outs = []
    for _ in range(2):
        dw = torch.zeros(96, 11, 11, 3, device=DEV)
        ops.conv_backward_weight(x, dy, dw, g)
        outs.append(dw)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


def test_alexnet_input_node_three_channels(monkeypatch):
    """The GPU net keeps AlexNet's input at 3 channels on 228-pixel rows and a training step
    matches the 4-channel layout's (CXXNET_CONV1_C3=0) loss and conv1 weight-gradient."""
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    out = []
    trs = []
    for c3 in ("1", "0"):
        monkeypatch.setenv("CXXNET_CONV1_C3", c3)
        pairs = load_conf("alexnet", [("batch_size", "8"), ("dev", "gpu"), ("eval_train", "0"), ("silent", "1"),
                                      ("update_period", "2")])
        tr = NetTrainer()
        for k, v in pairs:
            if not k.startswith("metric"):
                tr.set_param(k, v)
        tr.init_model()
        n0 = tr.net.nodes[0]
        assert (n0.cp, n0.data.shape[2]) == ((3, 228) if c3 == "1" else (4, 227))
        trs.append(tr)
    # same weights in both nets (the arenas differ in conv1's channel count)
    for ca, cb in zip(trs[0].net.connections, trs[1].net.connections):
        if ca.shared:
            continue
        for pa, pb in zip(ca.layer.params, cb.layer.params):
            if pa.shape == pb.shape:
                pb.w.copy_(pa.w.view(pb.w.shape))
            else:  # conv1 wmat [96][11][11][3] -> [96][11][11][4]
                pb.w.view(pb.shape).zero_()
                pb.w.view(pb.shape)[..., :3].copy_(pa.w.view(pa.shape))
    trs[1].net.arena.sync_shadow()
    for tr in trs:
        c, h, w = tr.net_cfg.input_shape
        g = torch.Generator().manual_seed(3)
        x = torch.randn(8, c, h, w, generator=g).to(DEV)
        y = torch.randint(0, 1000, (8, 1), generator=g).float().to(DEV)
        tr.net.set_input(x)
        tr.net.forward(False)
        torch.cuda.synchronize()
        fwd = (tr.net.nodes[1].data.float().clone(), tr.net.nodes[-1].data.float().clone())
        tr.update(DataBatch(x, y))
        torch.cuda.synchronize()
        conv1 = tr.net.connections[0].layer
        out.append(fwd + (conv1.w.g.view(96, 11, 11, -1)[..., :3].clone(),))
    # conv1's output agrees to bf16 rounding; the softmax output and conv1's weight-gradient pass
    # through 7 more bf16 layers each way and differ by their summation orders only
    # (test_conv1_three_channel_row_runs pins the kernels against fp32 torch)
    errs = [relerr(a, b) for a, b in zip(out[0], out[1])]
    assert errs[0] < 1e-2 and errs[1] < 6e-2 and errs[2] < 1e-1, errs


@pytest.fixture
def register_kernel_only():
    """Route every GEMM to the register-staged kernel (gemm_mfma.hip), whose MN-major tiles
    use the XOR-swizzled LDS image; the LDS-DMA kernel is restored afterwards."""
    from cxxnet_amd.ops import gemm
    gemm.set_glds(False)
    yield
    gemm.set_glds(True)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_backward_weight_register_kernel(case, register_kernel_only):
    test_conv_backward_weight(case)


@pytest.mark.parametrize("B,nin,nout", FC_CASES)
def test_fc_register_kernel(B, nin, nout, register_kernel_only):
    test_fc(B, nin, nout)


@pytest.mark.parametrize("relu,k,s,p,H", [(False, 3, 2, 0, 27), (True, 3, 2, 0, 28), (False, 3, 1, 1, 14),
                                          (False, 2, 2, 0, 28)])
def test_pool_tie_all(relu, k, s, p, H):
    """pool_tie = all kernel vs the CPU value-compare unpool, on data with many exact ties
    (values quantized to a few levels) and even sizes whose last windows run past the edge."""
    N, C = 2, 16
    g = torch.Generator().manual_seed(H + k)
    x = (torch.randint(-2, 3, (N, H, H, C), generator=g).float() * 0.5)
    Ho = ops.pool_out_size(H, k, s, p)
    y = torch.empty(N, Ho, Ho, C)
    ops.pool_forward(x, y, None, k, k, s, p, "max", relu)
    dy = rnd(N, Ho, Ho, C, seed=41)
    dx_ref = torch.empty_like(x)
    ops.pool_backward_tie_all(x, y, dy, dx_ref, k, k, s, p, relu=relu)
    xd = x.to(DEV, torch.bfloat16)
    yd = torch.empty(N, Ho, Ho, C, dtype=torch.bfloat16, device=DEV)
    ops.pool_forward(xd, yd, None, k, k, s, p, "max", relu)
    dx = torch.empty_like(xd)
    ops.pool_backward_tie_all(xd, yd, dy.to(DEV, torch.bfloat16), dx, k, k, s, p, relu=relu)
    torch.cuda.synchronize()
    assert torch.equal(yd.float().cpu(), y)
    assert relerr(dx, dx_ref) < 1e-2


@pytest.mark.parametrize("mode,k,s,H", [("max", 3, 2, 28), ("max", 2, 2, 28), ("max", 3, 2, 56), ("max", 3, 1, 14),
                                        ("avg", 3, 2, 28), ("avg", 2, 2, 56)])
@pytest.mark.parametrize("fused_relu", [False, True])
def test_pool_rows_even_sizes_and_relu_state(mode, k, s, H, fused_relu):
    """The production fast paths (pool_fwd_rows / pool_bwd_rows): even H/W, so the last window
    runs past the edge (GoogLeNet 112/56/28), and -- max mode after a fused conv+relu -- relu'
    read from bit 7 of the forward's argmax offsets (relu = 2, no dbias)."""
    N, C = 2, 64
    p = 1 if s == 1 else 0
    x = rnd(N, H, H, C, seed=51)
    if fused_relu:
        x = x.clamp_min(0)
    Ho = ops.pool_out_size(H, k, s, p)
    dy = rnd(N, Ho, Ho, C, seed=52)
    y_ref = torch.empty(N, Ho, Ho, C)
    st_ref = torch.empty(N, Ho, Ho, C, dtype=torch.uint8)
    ops.pool_forward(x, y_ref, st_ref, k, k, s, p, mode, False)
    dx_ref = torch.empty_like(x)
    ops.pool_backward(x, st_ref, dy, dx_ref, k, k, s, p, mode, fused_relu)
    xd = x.to(DEV, torch.bfloat16)
    y = torch.empty(N, Ho, Ho, C, dtype=torch.bfloat16, device=DEV)
    st = torch.empty(N, Ho, Ho, C, dtype=torch.uint8, device=DEV)
    mark = fused_relu and mode == "max"
    ops.pool_forward(xd, y, st, k, k, s, p, mode, False, mark_mask=mark)
    dx = torch.empty_like(xd)
    relu = (2 if mark else 1) if fused_relu else 0
    ops.pool_backward(xd, st, dy.to(DEV, torch.bfloat16), dx, k, k, s, p, mode, relu)
    torch.cuda.synchronize()
    assert relerr(y, y_ref) < 1e-2
    assert relerr(dx, dx_ref) < 2e-2


def test_bias_grad_multi_matches_single():
    """The deferred one-launch bias gradients (colsum_multi): conv-like (many rows, few
    channels), fc-like (few rows, 4096 channels: several 512-channel chunks per block) and a
    ragged C (falls back to the scalar kernel)."""
    shapes = [(200704, 64), (256, 4096), (43264, 384), (1000, 20)]
    items, refs = [], []
    for k, (r, c) in enumerate(shapes):
        dy = rnd(r, c, seed=60 + k).to(DEV, torch.bfloat16)
        db = torch.full((c,), 0.25, device=DEV)
        items.append((dy, db))
        refs.append(0.25 + dy.float().sum(0))
    ops.bias_grad_multi(items)
    torch.cuda.synchronize()
    for (_, db), ref in zip(items, refs):
        assert relerr(db, ref) < 1e-3


def test_bias_grad_masked_pool_offsets():
    """Masked colsum segments (the bias gradient of a conv in front of a max-pool, summed from
    the pool's output gradient): entries whose offset byte has bit 7 (relu' = 0) count as 0;
    mixed masked / unmasked segments in one launch, and the single-tensor entry point."""
    shapes = [(186624, 96), (43264, 256), (1000, 24)]
    items, refs = [], []
    for k, (r, c) in enumerate(shapes):
        dy = rnd(r, c, seed=80 + k).to(DEV, torch.bfloat16)
        g = torch.Generator().manual_seed(90 + k)
        off = torch.randint(0, 9, (r, c), generator=g, dtype=torch.uint8)
        off |= (torch.rand(r, c, generator=g) < 0.4).to(torch.uint8) * 128
        off = off.to(DEV)
        db = torch.full((c,), 0.5, device=DEV)
        m = off if k != 1 else None
        items.append((dy, db, m))
        keep = (off < 128).float() if m is not None else torch.ones(r, c, device=DEV)
        refs.append(0.5 + (dy.float() * keep).sum(0))
    ops.bias_grad_multi(items)
    torch.cuda.synchronize()
    for (_, db, _), ref in zip(items, refs):
        assert relerr(db, ref) < 1e-3
    dy, db, m = items[0][0], torch.zeros(96, device=DEV), items[0][2]
    ops.bias_grad(dy, db, m)
    assert relerr(db, refs[0] - 0.5) < 1e-3


def test_pool_fused_conv_bias_grad_matches_unfused():
    """conv -> relu -> max-pool: the conv's bias gradient taken by the pool from its output
    gradient (NeuralNet._fuse_pool_bias) equals the conv's own column sum of its dy."""
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer

    grads = []
    for fused in (True, False):
        # update_period 2: the first update() is forward + backward only (gradients kept)
        pairs = load_conf("alexnet", [("batch_size", "16"), ("dev", "gpu"), ("eval_train", "0"), ("silent", "1"),
                                      ("update_period", "2")])
        tr = NetTrainer()
        for k, v in pairs:
            if not k.startswith("metric"):
                tr.set_param(k, v)
        tr.init_model()
        pools = [c.layer for c in tr.net.connections if getattr(c.layer, "bias_of", None) is not None]
        assert len(pools) == 3  # conv1, conv2, conv5 sit in front of max-pools
        convs = [p.bias_of for p in pools]
        if not fused:
            for p in pools:
                p.bias_of = None
        c, h, w = tr.net_cfg.input_shape
        g = torch.Generator().manual_seed(5)
        x = torch.randn(16, c, h, w, generator=g).to(DEV)
        y = torch.randint(0, 1000, (16, 1), generator=g).float().to(DEV)
        tr.update(DataBatch(x, y))
        torch.cuda.synchronize()
        grads.append([cv.b.g.clone() for cv in convs])
    for a, b in zip(*grads):
        assert b.abs().max().item() > 0
        assert relerr(a, b) < 1e-2, relerr(a, b)


def test_lrn_fused_conv_bias_grad_matches_unfused():
    """GoogLeNet conv2 -> relu -> norm2: conv2's bias gradient summed by the LRN backward
    (NeuralNet._fuse_lrn_bias) equals the column-sum pass over conv2's output gradient."""
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer

    grads = []
    for fused in (True, False):
        pairs = load_conf("inception_v1", [("batch_size", "8"), ("dev", "gpu"), ("eval_train", "0"),
                                           ("silent", "1"), ("update_period", "2")])
        tr = NetTrainer()
        for k, v in pairs:
            if not k.startswith("metric"):
                tr.set_param(k, v)
        tr.init_model()
        lrns = [c.layer for c in tr.net.connections
                if type(c.layer).__name__ == "LRNLayer" and c.layer.bias_of is not None]
        assert len(lrns) == 1
        conv = lrns[0].bias_of
        if not fused:
            lrns[0].bias_of = None
        c, h, w = tr.net_cfg.input_shape
        g = torch.Generator().manual_seed(6)
        x = torch.randn(8, c, h, w, generator=g).to(DEV)
        y = torch.randint(0, 1000, (8, 1), generator=g).float().to(DEV)
        tr.update(DataBatch(x, y))
        torch.cuda.synchronize()
        grads.append(conv.b.g.clone())
    assert grads[1].abs().max().item() > 0
    # (the column sums cancel heavily: bf16 roundings of dx that differ in the last bit between
    # the two LRN kernels show at the 1e-3 level, as in the pool test above)
    assert relerr(grads[0], grads[1]) < 1e-2, relerr(grads[0], grads[1])


def test_concat_channels_one_launch():
    """ch_concat forward gather and backward scatter (relu' on the masked inputs) in one
    launch, against per-input slicing."""
    shapes = [64, 128, 32, 24]
    ins = [rnd(3, 7, 5, c, seed=70 + k).to(DEV, torch.bfloat16) for k, c in enumerate(shapes)]
    ins[1] = ins[1].clamp_min(0)  # relu(z) of a fused producer
    out = torch.empty(3, 7, 5, sum(shapes), dtype=torch.bfloat16, device=DEV)
    assert ops.concat_channels(ins, out)
    torch.cuda.synchronize()
    assert torch.equal(out, torch.cat(ins, -1))
    g = rnd(3, 7, 5, sum(shapes), seed=80).to(DEV, torch.bfloat16)
    acts = [t.clone() for t in ins]
    assert ops.concat_channels(ins, g, backward=True, mask={1})
    torch.cuda.synchronize()
    off = 0
    for k, c in enumerate(shapes):
        ref = g[..., off:off + c]
        if k == 1:
            ref = torch.where(acts[1] > 0, ref, torch.zeros_like(ref))
        assert torch.equal(ins[k], ref), k
        off += c


def test_conv_weight_flip_multi_matches_single():
    """One launch flips every conv layer's weights exactly as the per-layer kernel does."""
    from cxxnet_amd import native
    from cxxnet_amd.ops import gemm as G
    torch.manual_seed(5)
    geos = [ConvGeom(2, 13, 13, 384, 13, 13, 256, 3, 3, 1, 1, 1, 2), ConvGeom(2, 27, 27, 96, 27, 27, 256, 5, 5, 1, 2, 2, 2),
            ConvGeom(2, 28, 28, 192, 28, 28, 64, 1, 1, 1, 0, 0, 1), ConvGeom(2, 7, 7, 8, 7, 7, 16, 3, 3, 1, 1, 1, 1),
            ConvGeom(2, 7, 7, 12, 7, 7, 20, 3, 3, 1, 1, 1, 1),  # channels not multiples of 8: 2-byte path
            ConvGeom(2, 14, 14, 160, 14, 14, 72, 3, 3, 1, 1, 1, 1)]  # partial 64 x 64 tiles, 16-byte path
    items, refs = [], []
    for g in geos:
        w = torch.randn(g.Cout, g.KH, g.KW, g.cg_in, device=DEV).to(torch.bfloat16)
        wt = torch.empty_like(w)
        ref = torch.empty_like(w)
        native.check(native.kernels().cxn_conv_weight_flip(w.data_ptr(), ref.data_ptr(), g.groups, g.cg_out, g.KH,
                                                           g.KW, g.cg_in, G._stream()), "flip")
        items.append((w, wt, g))
        refs.append(ref)
    G.conv_weight_flip_multi(items)
    torch.cuda.synchronize()
    for (_, wt, _), ref in zip(items, refs):
        assert torch.equal(wt, ref)


@pytest.mark.parametrize("H,p", [(28, 1), (14, 1), (7, 1), (9, 0), (13, 1), (6, 2)])
@pytest.mark.parametrize("relu", [0, 1, 2])
def test_pool_stride1_3x3_strips(H, p, relu):
    """Stride-1 3x3 max pooling on row strips (pool_fwd_s1k3 / pool_bwd_s1k3, GoogLeNet's
    inception pool branches): outputs, first-max offsets (on data with many exact ties) and
    data-gradients against the CPU executor, for strip-ragged heights, pads 0-2 and the three
    relu modes (2 = relu' from the offsets' bit 7)."""
    N, C, k, s = 3, 24, 3, 1
    g = torch.Generator().manual_seed(100 * H + p + relu)
    x = torch.randint(-3, 4, (N, H, H + 1, C), generator=g).float() * 0.25
    if relu == 2:
        x = x.clamp_min(0)  # fused conv -> relu producer
    Ho = ops.pool_out_size(H, k, s, p)
    Wo = ops.pool_out_size(H + 1, k, s, p)
    dy = rnd(N, Ho, Wo, C, seed=H)
    y_ref = torch.empty(N, Ho, Wo, C)
    st_ref = torch.empty(N, Ho, Wo, C, dtype=torch.uint8)
    ops.pool_forward(x, y_ref, st_ref, k, k, s, p, "max", relu == 1)
    dx_ref = torch.empty_like(x)
    ops.pool_backward(x, st_ref, dy, dx_ref, k, k, s, p, "max", relu > 0)
    xd = x.to(DEV, torch.bfloat16)
    y = torch.empty(N, Ho, Wo, C, dtype=torch.bfloat16, device=DEV)
    st = torch.empty(N, Ho, Wo, C, dtype=torch.uint8, device=DEV)
    ops.pool_forward(xd, y, st, k, k, s, p, "max", relu == 1, mark_mask=relu == 2)
    dx = torch.empty_like(xd)
    ops.pool_backward(xd, st, dy.to(DEV, torch.bfloat16), dx, k, k, s, p, "max", relu)
    torch.cuda.synchronize()
    assert torch.equal(y.float().cpu(), y_ref)
    assert torch.equal(st.cpu() & 0x7F, st_ref)
    assert relerr(dx, dx_ref) < 1e-2


@pytest.mark.parametrize("H,W,p", [(55, 55, 0), (27, 27, 0), (13, 14, 0), (28, 28, 1), (9, 8, 1), (7, 7, 2)])
@pytest.mark.parametrize("relu", [0, 1, 2])
def test_pool_bwd_stride2_3x3_cells(H, W, p, relu):
    """3x3 stride-2 max-unpool on 2x2 input cells (pool_bwd_s2k3, AlexNet / GoogLeNet pools):
    against the CPU executor for odd / even / non-square sizes, pads 0-2 and the three relu
    modes, and bitwise against the one-pixel-per-thread kernel (kernel variant 0)."""
    from cxxnet_amd import native
    N, C, k, s = 2, 40, 3, 2
    g = torch.Generator().manual_seed(10 * H + W + p + relu)
    x = torch.randint(-3, 4, (N, H, W, C), generator=g).float() * 0.25
    if relu == 2:
        x = x.clamp_min(0)
    Ho, Wo = ops.pool_out_size(H, k, s, p), ops.pool_out_size(W, k, s, p)
    dy = rnd(N, Ho, Wo, C, seed=H + W)
    y_ref = torch.empty(N, Ho, Wo, C)
    st_ref = torch.empty(N, Ho, Wo, C, dtype=torch.uint8)
    ops.pool_forward(x, y_ref, st_ref, k, k, s, p, "max", relu == 1)
    dx_ref = torch.empty_like(x)
    ops.pool_backward(x, st_ref, dy, dx_ref, k, k, s, p, "max", relu > 0)
    xd = x.to(DEV, torch.bfloat16)
    y = torch.empty(N, Ho, Wo, C, dtype=torch.bfloat16, device=DEV)
    st = torch.empty(N, Ho, Wo, C, dtype=torch.uint8, device=DEV)
    ops.pool_forward(xd, y, st, k, k, s, p, "max", relu == 1, mark_mask=relu == 2)
    dyd = dy.to(DEV, torch.bfloat16)
    out = []
    for v in (1, 0):
        native.check(native.kernels().cxn_set_kernel_variant(0, v), "variant")
        dx = torch.full_like(xd, 7.0)  # every pixel must be written
        ops.pool_backward(xd, st, dyd, dx, k, k, s, p, "max", relu)
        out.append(dx)
    native.check(native.kernels().cxn_set_kernel_variant(0, 1), "variant")
    torch.cuda.synchronize()
    assert torch.equal(out[0], out[1])
    assert relerr(out[0], dx_ref) < 1e-2


@pytest.mark.parametrize("geo_args,mask", [((4, 13, 13, 384, 13, 13, 384, 3, 3, 1, 1, 1, 2), True),
                                           ((2, 28, 28, 64, 28, 28, 96, 3, 3, 1, 1, 1, 1), False),
                                           ((2, 14, 14, 48, 14, 14, 64, 5, 5, 1, 2, 2, 1), True)])
def test_conv_dgrad_epilogue_bias_sum(geo_args, mask):
    """The data-gradient GEMM's EPI_BF16_DB epilogue: dx as the plain epilogue writes it, and
    dbias += column sums of the stored (relu'-masked) dx."""
    from cxxnet_amd.ops.gemm import ConvGeom
    g = ConvGeom(*geo_args)
    dy = rnd(g.N, g.Ho, g.Wo, g.Cout, seed=7).to(DEV, torch.bfloat16)
    w = (rnd(g.Cout, g.KH, g.KW, g.cg_in, seed=8) * 0.05).to(DEV, torch.bfloat16)
    z = rnd(g.N, g.H, g.W, g.C, seed=9).to(DEV, torch.bfloat16)
    dx_ref = z.clone() if mask else torch.empty_like(z)
    ops.conv_backward_data(dy, w, dx_ref, g, mask_relu=mask)
    dx = z.clone() if mask else torch.empty_like(z)
    db = torch.full((g.C,), 0.25, device=DEV)
    fused = ops.conv_backward_data(dy, w, dx, g, mask_relu=mask, dbias=db)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx_ref)
    ref = 0.25 + dx_ref.float().reshape(-1, g.C).sum(0)
    if fused:
        assert relerr(db, ref) < 1e-3
    else:
        assert torch.equal(db, torch.full_like(db, 0.25))


@pytest.mark.parametrize("model,batch,nfused", [("alexnet", 16, 2), ("vgg16", 2, 8)])
def test_dgrad_fused_bias_grads_match_unfused(monkeypatch, model, batch, nfused):
    """conv -> relu -> conv: the lower conv's bias gradient from the upper conv's data-gradient
    epilogue (NeuralNet._fuse_dgrad_bias, every eligible layer) equals the column-sum pass, on
    AlexNet (conv3, conv4: the direct kernels) and VGG-16 (the halo and LDS-DMA epilogues)."""
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer

    grads = []
    for fused in ("1", "0"):
        monkeypatch.setenv("CXXNET_DGRAD_BIAS", fused)
        pairs = load_conf(model, [("batch_size", str(batch)), ("dev", "gpu"), ("eval_train", "0"), ("silent", "1"),
                                  ("update_period", "2")])
        tr = NetTrainer()
        for k, v in pairs:
            if not k.startswith("metric"):
                tr.set_param(k, v)
        tr.init_model()
        below = [c.layer.bias_below for c in tr.net.connections if getattr(c.layer, "bias_below", None) is not None]
        assert len(below) == (nfused if fused == "1" else 0)
        c, h, w = tr.net_cfg.input_shape
        g = torch.Generator().manual_seed(6)
        x = torch.randn(batch, c, h, w, generator=g).to(DEV)
        y = torch.randint(0, 1000, (batch, 1), generator=g).float().to(DEV)
        tr.update(DataBatch(x, y))
        torch.cuda.synchronize()
        grads.append([cn.layer.b.g.clone() for cn in tr.net.connections
                      if type(cn.layer).__name__ == "ConvolutionLayer" and cn.layer.b is not None])
    for a, b in zip(*grads):
        assert b.abs().max().item() > 0
        assert relerr(a, b) < 1e-2, relerr(a, b)


def test_dgrad_bias_auto_with_siblings_matches_unfused(monkeypatch):
    """GoogLeNet with the sibling 1x1 groups on and the dgrad-bias fusion in "auto" mode at a 0 MB
    threshold (every eligible conv): no sibling member becomes a bias target (the group sums its
    biases over its shared buffer -- a member's bias would count twice), and every conv bias
    gradient matches the run without the fusion."""
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer

    grads = []
    for mode in ("auto", "0"):
        monkeypatch.setenv("CXXNET_DGRAD_BIAS", mode)
        monkeypatch.setenv("CXXNET_DGRAD_BIAS_MIN_MB", "0")
        pairs = load_conf("inception_v1", [("batch_size", "4"), ("dev", "gpu"), ("eval_train", "0"),
                                           ("silent", "1"), ("update_period", "2")])
        tr = NetTrainer()
        for k, v in pairs:
            if not k.startswith("metric"):
                tr.set_param(k, v)
        tr.init_model()
        assert tr.net.sib_groups  # the sibling groups stay on
        below = [c.layer.bias_below for c in tr.net.connections if getattr(c.layer, "bias_below", None) is not None]
        assert not any(b.sib is not None or b.sib_member for b in below)
        if mode == "auto":
            assert below  # conv2_reduce -> conv2 at least
        c, h, w = tr.net_cfg.input_shape
        g = torch.Generator().manual_seed(8)
        x = torch.randn(4, c, h, w, generator=g).to(DEV)
        y = torch.randint(0, 1000, (4, 1), generator=g).float().to(DEV)
        tr.update(DataBatch(x, y))
        torch.cuda.synchronize()
        grads.append([(i, s.g.clone()) for i, s in tr.net.arena.specs if s.tag == "bias"])
    for (i, a), (j, b) in zip(*grads):
        assert i == j
        assert relerr(a, b) < 1e-2, (i, relerr(a, b))


FEWC_CASES = [
    # N, H, W, Cout, K, stride, pad, relu, bias, ldc_extra
    (2, 224, 224, 64, 3, 1, 1, True, True, 0),    # VGG conv1_1
    (2, 224, 224, 64, 7, 2, 3, True, True, 0),    # GoogLeNet conv1
    (3, 37, 53, 48, 5, 1, 2, False, True, 0),     # ragged width (last 16-pixel column partial)
    (2, 300, 300, 16, 3, 2, 0, True, False, 0),   # Wo > 256: two passes; no bias
    (1, 19, 23, 128, 8, 3, 1, True, True, 0),     # even kernel, stride 3, 128 channels
    (2, 33, 31, 32, 3, 1, 1, True, True, 64),     # channel slice of a wider buffer (ldc 96)
]


@pytest.mark.parametrize("case", FEWC_CASES)
def test_conv_fewc_forward(case):
    """Few-channel first-layer kernel (conv_fewc.hip) against the fp32 torch conv."""
    N, H, W, Cout, K, s, p, relu, use_b, extra = case
    geo = _geom(N, 4, H, W, Cout, K, s, p, 1)
    x = rnd(N, H, W, 4, seed=1)
    w = rnd(Cout, K, K, 4, scale=0.05, seed=2)
    b = rnd(Cout, scale=0.1, seed=3) if use_b else None
    y_ref = torch.empty(N, geo.Ho, geo.Wo, Cout)
    ops.conv_forward(x, w, b, y_ref, geo, relu=relu)
    full = torch.full((N, geo.Ho, geo.Wo, Cout + extra), 7.0, dtype=torch.bfloat16, device=DEV)
    y = full[..., :Cout]
    ran = ops.gemm.conv_forward_fewc(x.to(DEV, torch.bfloat16), w.to(DEV, torch.bfloat16),
                                     b.to(DEV) if b is not None else None, y, geo, relu=relu)
    torch.cuda.synchronize()
    assert ran, "the few-channel kernel did not take the shape"
    assert relerr(y, y_ref) < 2e-2
    if extra:
        assert bool((full[..., Cout:] == 7.0).all()), "wrote outside its channel slice"


@pytest.mark.parametrize("B,R,Cc", [(256, 36, 256), (256, 256, 36), (64, 49, 512), (70, 12, 20), (3, 36, 256)])
def test_transpose_batched_shapes(B, R, Cc):
    """ops.transpose: the per-item LDS kernel (AlexNet's flatten, both directions, B >= 64) and the
    tiled fallback (odd row counts, small batches) give the exact transpose."""
    x = torch.randn(B, R, Cc, device=DEV).to(torch.bfloat16)
    y = torch.empty(B, Cc, R, device=DEV, dtype=torch.bfloat16)
    ops.transpose(x, y, B, R, Cc)
    torch.cuda.synchronize()
    assert torch.equal(y, x.transpose(1, 2))
