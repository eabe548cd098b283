"""Correctness gate for the GEMM tile choices.

* every entry of the shipped tuning table (ops/glds_tune_gfx950.json) runs at its exact
  signature -- the kernels behind the published img/s numbers -- against an fp32 torch
  reference of the same op on the same bf16-rounded operands;
* every autotuning candidate tile (GLDS_CANDS + the register kernel) runs on one
  representative shape per op class against the same reference;
* the autotuner rejects a tile whose output is wrong however fast it is.
"""
import pytest
import torch
import torch.nn.functional as F

from cxxnet_amd import ops
from cxxnet_amd.ops import gemm
from cxxnet_amd.ops.gemm import ConvGeom, conv_out_size

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rnd(shape, scale, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV) * scale).to(torch.bfloat16)


def _relnorm(a, ref):
    a, ref = a.float(), ref.float()
    return ((a - ref).norm() / ref.norm().clamp_min(1e-30)).item()


def _geom(key):
    N, H, W, C, Cout, KH, KW, s, py, px, G = key
    Ho, Wo = conv_out_size(H, W, KH, KW, s, py, px)
    return ConvGeom(N, H, W, C, Ho, Wo, Cout, KH, KW, s, py, px, G)


def _w_nchw(w):
    return w.float().permute(0, 3, 1, 2)


def check_conv(op, key, tile=None):
    """Run conv op `op` (cf / cr / cd / cw) at signature `key` and return the norm-relative
    error against torch fp32.  `tile` forces a tile (None: the table / tuner choice)."""
    g = _geom(key)
    if tile is not None:
        gemm.set_glds(tile=tile)
    try:
        if op in ("cf", "cr"):
            x = _rnd((g.N, g.H, g.W, g.C), 1.0, 1)
            w = _rnd((g.Cout, g.KH, g.KW, g.cg_in), 0.05, 2)
            b = torch.randn(g.Cout, device=DEV) * 0.1
            y = torch.empty(g.N, g.Ho, g.Wo, g.Cout, dtype=torch.bfloat16, device=DEV)
            ops.conv_forward(x, w, b, y, g)
            ref = F.conv2d(x.float().permute(0, 3, 1, 2), _w_nchw(w), b, stride=g.stride,
                           padding=(g.pad_y, g.pad_x), groups=g.groups).permute(0, 2, 3, 1)
            return _relnorm(y, ref)
        if op == "cd":
            dy = _rnd((g.N, g.Ho, g.Wo, g.Cout), 1.0, 3)
            w = _rnd((g.Cout, g.KH, g.KW, g.cg_in), 0.05, 4)
            dx = torch.empty(g.N, g.H, g.W, g.C, dtype=torch.bfloat16, device=DEV)
            ops.conv_backward_data(dy, w, dx, g)
            ref = torch.nn.grad.conv2d_input((g.N, g.C, g.H, g.W), _w_nchw(w), dy.float().permute(0, 3, 1, 2),
                                             stride=g.stride, padding=(g.pad_y, g.pad_x),
                                             groups=g.groups).permute(0, 2, 3, 1)
            return _relnorm(dx, ref)
        if op in ("cw", "cws"):
            x = _rnd((g.N, g.H, g.W, g.C), 1.0, 5)
            dy = _rnd((g.N, g.Ho, g.Wo, g.Cout), 1.0, 6)
            dw = torch.zeros(g.Cout, g.KH, g.KW, g.cg_in, device=DEV)
            ops.conv_backward_weight(x, dy, dw, g)
            ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (g.Cout, g.cg_in, g.KH, g.KW),
                                              dy.float().permute(0, 3, 1, 2), stride=g.stride,
                                              padding=(g.pad_y, g.pad_x), groups=g.groups).permute(0, 2, 3, 1)
            return _relnorm(dw, ref)
        raise ValueError(op)
    finally:
        gemm.set_glds(tile=-1)


def check_fc(op, nin, nout, B, tile=None):
    if tile is not None:
        gemm.set_glds(tile=tile)
    try:
        x = _rnd((B, nin), 1.0, 7)
        w = _rnd((nout, nin), 0.02, 8)
        if op == "fc":
            b = torch.randn(nout, device=DEV) * 0.1
            y = torch.empty(B, nout, dtype=torch.bfloat16, device=DEV)
            ops.fc_forward(x, w, b, y)
            return _relnorm(y, x.float() @ w.float().t() + b)
        dy = _rnd((B, nout), 1.0, 9)
        dw = torch.empty(nout, nin, device=DEV)
        ops.fc_backward_weight(x, dy, dw, overwrite=True)
        return _relnorm(dw, dy.float().t() @ x.float())
    finally:
        gemm.set_glds(tile=-1)


def _table_cases():
    out = []
    for k in sorted(gemm._TUNE):
        parts = k.split("|")
        out.append(pytest.param(parts[0], tuple(int(v) for v in parts[1:]), id=k))
    return out


@pytest.mark.parametrize("op,sig", _table_cases())
def test_shipped_table_entry(op, sig):
    """The table's tile at the table's exact signature (no tile forcing: the lookup
    inside the op picks it, as in training)."""
    if op in ("cf", "cr", "cd", "cw", "cws"):
        if op == "cr":  # key: N, H, W, C, Cout, KH, KW, stride (no pad, one group)
            sig = sig + (0, 0, 1)
        err = check_conv(op, sig)
    elif op == "cwr":  # row-run weight-grad (few channels, conv1): key as "cr"
        err = check_conv("cw", sig + (0, 0, 1))
    elif op == "fc":
        _, nout, B, nin, _ = sig  # amode, a.rows = nout, b.rows = B, kdim = nin, ldc
        err = check_fc("fc", nin, nout, B)
    elif op == "fws":
        nin, nout, B = sig
        err = check_fc_sgd(nin, nout, B)
    elif op == "cfs":
        err = check_conv_split(sig)
    else:
        nin, nout, B = sig
        err = check_fc("fw", nin, nout, B)
    assert err < 1e-2, (op, sig, gemm._TUNE.get("|".join([op] + [str(v) for v in sig])), err)


def check_conv_split(sig):
    """Sibling 1x1 convs as one two-destination GEMM (key "cfs": N, H, W, C, Cout, split):
    channels [0, split) into a slice of a wider buffer, the rest into a second buffer."""
    N, H, W, C, Cout, split = sig
    x = _rnd((N, H, W, C), 1.0, 21)
    w = _rnd((Cout, 1, 1, C), 0.05, 22)
    b = torch.randn(Cout, device=DEV) * 0.1
    big = torch.zeros(N, H, W, split + 64, device=DEV, dtype=torch.bfloat16)
    y, y2 = big[..., 32:32 + split], torch.empty(N, H, W, Cout - split, device=DEV, dtype=torch.bfloat16)
    ops.gemm.conv_forward_split(x, w, b, y, y2, split, ConvGeom(N, H, W, C, H, W, Cout, 1, 1, 1, 0, 0, 1), relu=True)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b).clamp_min(0).permute(0, 2, 3, 1)
    return _relnorm(torch.cat([y.float(), y2.float()], -1), ref)


def check_fc_sgd(nin, nout, B):
    """The fc weight-gradient fused with the SGD step (table key "fws") against torch:
    m' = mom m - lr (dy^T x + wd w), w' = w + m'; returns the worse relative error of m' and w'."""
    x = _rnd((B, nin), 1.0, 11)
    dy = _rnd((B, nout), 1.0, 12)
    w = torch.randn(nout, nin, device=DEV) * 0.02
    m = torch.randn(nout, nin, device=DEV) * 0.01
    wb = w.to(torch.bfloat16)
    lr, wd, mom = 0.01, 5e-4, 0.9
    g = dy.float().t() @ x.float()
    m_ref = mom * m - lr * (g + wd * w)
    w_ref = w + m_ref
    assert ops.fc_backward_weight_sgd(x, dy, w, m, wb, lr, wd, mom, 0.0)
    return max(_relnorm(m, m_ref), _relnorm(w, w_ref), _relnorm(wb.float(), w_ref))


# one representative (non-table) shape per op class; each candidate tile is forced
REPS = {
    "cf": (16, 27, 27, 96, 256, 5, 5, 1, 2, 2, 2),
    "cd": (16, 13, 13, 256, 384, 3, 3, 1, 1, 1, 1),
    "cw": (16, 13, 13, 384, 256, 3, 3, 1, 1, 1, 2),
    "cr": (8, 227, 227, 4, 96, 11, 11, 4, 0, 0, 1),
}


@pytest.mark.parametrize("tile", list(gemm.GLDS_CANDS) + [gemm.REG])
@pytest.mark.parametrize("op", ["cf", "cd", "cw", "cr", "fc", "fw"])
def test_every_candidate_tile(op, tile):
    if op in ("cr", "fc", "fw") and tile == gemm.REG:
        pytest.skip("the register-kernel pseudo-tile is a candidate for conv fwd / dgrad / wgrad only")
    if op in REPS:
        err = check_conv(op, REPS[op], tile=tile)
    else:
        err = check_fc(op, 4096, 1000, 96, tile=tile)
    assert err < 1e-2, (op, tile, err)


def test_tuner_rejects_a_wrong_fast_tile(monkeypatch):
    """A candidate that writes garbage instantly must never be chosen."""
    calls = {}

    def run(tile, out):
        calls[tile] = calls.get(tile, 0) + 1
        if tile == 15:  # "fast" and wrong
            out.fill_(1.0)
            return True
        out.copy_(torch.arange(out.numel(), device=DEV, dtype=out.dtype).view_as(out))
        torch.cuda._sleep(200000)  # the correct tiles are slow
        return True

    out = torch.zeros(64, 64, device=DEV)
    gemm.TUNE_REJECTED.clear()
    monkeypatch.setattr(gemm, "GLDS_CANDS", (1, 15, 7))
    t = gemm._tuned_tile(("test-reject", 1), run, out, lambda: 1)
    assert t != 15
    assert any(k == "test-reject|1" and tl == 15 for k, tl, _ in gemm.TUNE_REJECTED)
    gemm._TUNE.pop("test-reject|1", None)


@pytest.mark.parametrize("tile", gemm.WGRAD_TILES)
@pytest.mark.parametrize("sig", [
    (4, 27, 27, 96, 96, 5, 5, 1, 2, 2, 1),     # 96 output channels: tile 6's exact fit
    (4, 14, 14, 480, 16, 1, 1, 1, 0, 0, 1),    # GoogLeNet 5x5-reduce: 16 channels (tile 7)
    (2, 28, 28, 32, 32, 5, 5, 1, 2, 2, 1),     # 32 channels, 5x5
    (2, 55, 55, 96, 256, 5, 5, 1, 2, 2, 2),    # grouped, 128 per group
])
def test_register_wgrad_tiles(tile, sig):
    """Every register-kernel weight-grad tile (split-K fp32 atomics) at a forced (tile, split)
    against torch, through the per-shape "cws" table entry the op looks up."""
    key = "|".join(["cws"] + [str(v) for v in sig])
    saved = gemm._TUNE.get(key)
    gemm._TUNE[key] = tile * 100000 + 3
    try:
        err = check_conv("cw", sig)
    finally:
        if saved is None:
            gemm._TUNE.pop(key, None)
        else:
            gemm._TUNE[key] = saved
    assert err < 1e-2, (tile, sig, err)
