"""Max-pool -> LRN fused (NeuralNet._fuse_pool_lrn; ops.pool_lrn_forward / lrn_pool_backward) on
AlexNet against the separate layers (CXXNET_FUSE_POOL_LRN=0), both in deterministic mode:
after one training step every
parameter is bitwise the same, except the biases of conv1 / conv2, whose gradient the fused
backward sums in another order (fp32 partial rows instead of the column-sum pass); and the
fused kernels' outputs against fp32 torch pooling + LRN."""
import pytest
import torch
import torch.nn.functional as F

from cxxnet_amd import ops
from cxxnet_amd.io.data import DataBatch
from cxxnet_amd.models import load_conf
from cxxnet_amd.nnet import NetTrainer

pytestmark = pytest.mark.gpu


def _alexnet(batch, fuse, monkeypatch):
    monkeypatch.setenv("CXXNET_FUSE_POOL_LRN", fuse)
    tr = NetTrainer()
    base = [(k, v) for k, v in load_conf("alexnet", []) if not k.startswith("metric")]
    # deterministic: the split-K weight-gradients' fp32 atomics would differ run to run
    for k, v in base + [("batch_size", str(batch)), ("dev", "gpu"), ("eval_train", "0"), ("silent", "1"),
                        ("seed", "11"), ("deterministic", "1")]:
        tr.set_param(k, v)
    tr.init_model()
    pools = [c.layer for c in tr.net.connections if type(c.layer).__name__ == "PoolingLayer"]
    assert sum(p.fused_lrn is not None for p in pools) == (2 if fuse == "1" else 0)
    return tr


def test_alexnet_step_fused_pool_lrn_matches(monkeypatch):
    B = 16
    g = torch.Generator().manual_seed(2)
    x = torch.randn(B, 3, 227, 227, generator=g).cuda()
    y = torch.randint(0, 1000, (B, 1), generator=g).float().cuda()
    res = {}
    for fuse in ("0", "1"):
        tr = _alexnet(B, fuse, monkeypatch)
        tr.update(DataBatch(x, y))
        torch.cuda.synchronize()
        res[fuse] = {(li, s.tag): s.w.clone() for li, s in tr.net.arena.specs}
        names = {li: tr.net.connections[li].layer for li, _ in tr.net.arena.specs}
    for key, a in res["0"].items():
        b = res["1"][key]
        li, tag = key
        if tag == "bias" and type(names[li]).__name__ == "ConvolutionLayer":
            assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), key
        else:
            assert torch.equal(a, b), key


@pytest.mark.parametrize("H,C,relu", [(55, 96, 2), (55, 96, 6), (27, 256, 6), (27, 256, 2), (13, 64, 0), (8, 32, 6)])
def test_pool_lrn_kernels_vs_torch(H, C, relu):
    N, n, alpha, beta, k = 3, 5, 1e-3, 0.75, 1.0
    torch.manual_seed(H)
    x = torch.randn(N, H, H, C, device="cuda").clamp_min(0).to(torch.bfloat16)  # relu'd conv output
    Ho = min(H - 2, H - 1) // 2 + 1
    P = torch.empty(N, Ho, Ho, C, device="cuda", dtype=torch.bfloat16)
    st = torch.empty(N, Ho, Ho, C, device="cuda", dtype=torch.uint8)
    Y = torch.empty_like(P)
    assert ops.pool_lrn_forward(x, P, st, Y, relu, n, alpha, beta, k)
    xr = x.float().permute(0, 3, 1, 2)
    pr = F.max_pool2d(xr, 3, 2, ceil_mode=True)
    assert torch.equal(P.float().permute(0, 3, 1, 2), pr)
    yr = F.local_response_norm(P.float().permute(0, 3, 1, 2), n, alpha=alpha, beta=beta, k=k)
    assert ((Y.float().permute(0, 3, 1, 2) - yr).norm() / yr.norm()).item() < 1e-2
    # backward against autograd of the fp32 reference pair, the gradient masked by relu' of the max
    dY = torch.randn_like(Y)
    dx = torch.empty_like(x)
    db = torch.zeros(C, device="cuda")
    rows = ops.lrn_pool_backward_rows(x.shape, P.shape, n)
    part = torch.empty(rows, C, device="cuda")
    assert ops.lrn_pool_backward(P, dY, st, dx, int((relu & 2) != 0), n, alpha, beta, k, dbias=db, part=part)
    xv = xr.clone().requires_grad_(True)
    pv = F.max_pool2d(xv, 3, 2, ceil_mode=True)
    pv.retain_grad()
    yv = F.local_response_norm(pv, n, alpha=alpha, beta=beta, k=k)
    yv.backward(dY.float().permute(0, 3, 1, 2))
    gx = xv.grad
    gp = pv.grad
    if relu & 2:
        gx = gx * (xr > 0).float()
        gp = gp * (pv.detach() > 0).float()
    err = ((dx.float().permute(0, 3, 1, 2) - gx).norm() / gx.norm()).item()
    assert err < 2e-2, err
    dbr = gp.sum((0, 2, 3))
    assert ((db - dbr).norm() / dbr.norm()).item() < 2e-2


def test_pool_lrn_bias_sum_deterministic():
    """Deterministic mode: the fused backward's conv-bias sum (per-block rows in a fixed order,
    then one ordered pass over the rows) is bitwise repeatable; 64 images of AlexNet pool1 give
    448 partial rows (more than one 256-row chunk)."""
    from cxxnet_amd.ops import gemm
    N, H, C, n = 64, 55, 96, 5
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device="cuda").clamp_min(0).to(torch.bfloat16)
    Ho = (H - 3) // 2 + 1
    P = torch.empty(N, Ho, Ho, C, device="cuda", dtype=torch.bfloat16)
    st = torch.empty(N, Ho, Ho, C, device="cuda", dtype=torch.uint8)
    Y = torch.empty_like(P)
    assert ops.pool_lrn_forward(x, P, st, Y, 2, n, 1e-4, 0.75, 1.0)
    dY = torch.randn_like(Y)
    dx = torch.empty_like(x)
    rows = ops.lrn_pool_backward_rows(x.shape, P.shape, n)
    assert rows > 256
    part = torch.empty(rows, C, device="cuda")
    gemm.set_deterministic(True)
    out = []
    for _ in range(3):
        db = torch.zeros(C, device="cuda")
        assert ops.lrn_pool_backward(P, dY, st, dx, 1, n, 1e-4, 0.75, 1.0, dbias=db, part=part)
        out.append(db)
    assert torch.equal(out[0], out[1]) and torch.equal(out[0], out[2])


def test_pool_lrn_integer_key_max_matches_float_compare():
    """The non-negative-input path (flag 4: integer keys) against the float-compare path on
    inputs full of ties and signed zeros: same maxima, same first-max offsets, same LRN."""
    N, H, C, n = 4, 27, 64, 5
    g = torch.Generator(device="cuda").manual_seed(3)
    vals = torch.tensor([0.0, -0.0, 1.0, 2.0, 0.5], device="cuda")
    x = vals[torch.randint(0, 5, (N, H, H, C), generator=g, device="cuda")].to(torch.bfloat16)
    Ho = (H - 3) // 2 + 1
    out = {}
    for flags in (2, 6):
        P = torch.empty(N, Ho, Ho, C, device="cuda", dtype=torch.bfloat16)
        st = torch.empty(N, Ho, Ho, C, device="cuda", dtype=torch.uint8)
        Y = torch.empty_like(P)
        assert ops.pool_lrn_forward(x, P, st, Y, flags, n, 1e-4, 0.75, 1.0)
        out[flags] = (P.float(), st.clone(), Y.float())
    assert torch.equal(out[2][0], out[6][0])
    assert torch.equal(out[2][1], out[6][1])
    assert torch.equal(out[2][2], out[6][2])
