"""Sibling 1x1 convs of GoogLeNet's inception modules as one GEMM per direction
(NeuralNet._fuse_siblings, ops.gemm.conv_forward_split) against the unfused layers
(CXXNET_FUSE_SIBLINGS=0): every module fused, the same training step to bf16 accuracy, and the
two-destination GEMM against fp32 torch."""
import pytest
import torch
import torch.nn.functional as F

from cxxnet_amd import ops
from cxxnet_amd.io.data import DataBatch
from cxxnet_amd.models import load_conf
from cxxnet_amd.nnet import NetTrainer
from cxxnet_amd.ops.gemm import ConvGeom

pytestmark = pytest.mark.gpu


def _net(fuse, monkeypatch, batch=8):
    monkeypatch.setenv("CXXNET_FUSE_SIBLINGS", fuse)
    tr = NetTrainer()
    base = [(k, v) for k, v in load_conf("inception_v1", []) if not k.startswith("metric")]
    for k, v in base + [("batch_size", str(batch)), ("dev", "gpu"), ("eval_train", "0"), ("silent", "1"),
                        ("seed", "5"), ("deterministic", "1")]:
        tr.set_param(k, v)
    tr.init_model()
    return tr


def test_inception_step_fused_siblings_match(monkeypatch):
    B = 8
    g = torch.Generator().manual_seed(4)
    x = torch.randn(B, 3, 224, 224, generator=g).cuda()
    y = torch.randint(0, 1000, (B, 1), generator=g).float().cuda()
    res = {}
    trs = {fuse: _net(fuse, monkeypatch, B) for fuse in ("0", "1")}
    assert len(trs["0"].net.sib_groups) == 0 and len(trs["1"].net.sib_groups) == 9
    # the same initial weights (the arena order, and so the init draw order, differs)
    src = {(li, s.tag): s.w for li, s in trs["0"].net.arena.specs}
    for li, s in trs["1"].net.arena.specs:
        s.w.copy_(src[(li, s.tag)])
    trs["1"].net.arena.sync_shadow()
    for fuse, tr in trs.items():
        w0 = {(li, s.tag): s.w.clone() for li, s in tr.net.arena.specs}
        tr.update(DataBatch(x, y))
        torch.cuda.synchronize()
        res[fuse] = {(li, s.tag): (s.w - w0[(li, s.tag)]) for li, s in tr.net.arena.specs}
    worst = 0.0
    for key, d0 in res["0"].items():
        d1 = res["1"][key]
        err = ((d1 - d0).norm() / d0.norm().clamp_min(1e-12)).item()
        worst = max(worst, err)
        assert err < 5e-2, (key, err)
    assert worst < 5e-2


@pytest.mark.parametrize("split,cout,ldc", [(64, 176, 256), (128, 320, 128), (16, 40, 16)])
def test_conv_forward_split_vs_torch(split, cout, ldc):
    N, H, C = 4, 14, 192
    torch.manual_seed(split)
    x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
    w = (torch.randn(cout, 1, 1, C, device="cuda") * 0.05).to(torch.bfloat16)
    b = torch.randn(cout, device="cuda") * 0.1
    big = torch.full((N, H, H, ldc + split), 7.0, device="cuda", dtype=torch.bfloat16)
    y = big[..., 8:8 + split] if ldc + split > split + 8 else big[..., :split]
    y2 = torch.empty(N, H, H, cout - split, device="cuda", dtype=torch.bfloat16)
    g = ConvGeom(N, H, H, C, H, H, cout, 1, 1, 1, 0, 0, 1)
    ops.gemm.conv_forward_split(x, w, b, y, y2, split, g, relu=True)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b).clamp_min(0).permute(0, 2, 3, 1)
    got = torch.cat([y.float(), y2.float()], -1)
    assert ((got - ref).norm() / ref.norm()).item() < 1e-2
