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


def test_fused_model_file_is_byte_identical(monkeypatch):
    """Sibling groups change only the arena layout: from the same seed the fused net draws the
    same initial weights, writes the same model file byte for byte, and loads the unfused
    net's file back to the same bytes."""
    plain, fused = _net("0", monkeypatch), _net("1", monkeypatch)
    assert len(fused.net.sib_groups) == 9
    a, b = plain.save_model(), fused.save_model()
    assert a == b
    other = _net("1", monkeypatch)
    other.load_model(a)
    assert other.save_model() == a


@pytest.mark.parametrize("tile", [1, 7, 38, 79])
def test_dgrad_with_added_gradient_vs_torch(tile):
    """ops.gemm.conv_backward_data_add (the split's sum folded into a sibling group's
    data-gradient GEMM): dx = relu'(x) * (conv_transpose(dy, w) + add) on a forced LDS-DMA tile,
    against fp32 torch."""
    from cxxnet_amd.ops import gemm as G
    N, H, C, K = 4, 14, 192, 176
    torch.manual_seed(tile)
    dy = torch.randn(N, H, H, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(K, 1, 1, C, device="cuda") * 0.05).to(torch.bfloat16)
    add = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
    act = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)  # relu output where > 0
    g = ConvGeom(N, H, H, C, H, H, K, 1, 1, 1, 0, 0, 1)
    for mask in (False, True):
        dx = act.clone()
        G.set_glds(True, tile)
        try:
            assert G.conv_backward_data_add(dy, w, dx, add, g, torch.empty_like(w), mask_relu=mask)
        finally:
            G.set_glds(True, -1)
        assert G.LAST_GLDS[0] == tile
        ref = torch.einsum("nhwk,kc->nhwc", dy.float(), w.float().view(K, C)) + add.float()
        if mask:
            ref = ref * (act.float() > 0)
        assert ((dx.float() - ref).norm() / ref.norm()).item() < 1e-2, (tile, mask)


def test_split_sum_folded_in_training(monkeypatch):
    """GoogLeNet at batch 16: after the first steps tuned the data-gradient signatures, the
    splits of the sibling modules skip their sums (folded into the groups' GEMMs), and the
    step still matches the unfolded one (CXXNET_FOLD_SPLIT_SUM=0)."""
    B = 16
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, 3, 224, 224, generator=g).cuda()
    y = torch.randint(0, 1000, (B, 1), generator=g).float().cuda()
    res, trs = {}, {}
    for fold in ("0", "1"):
        monkeypatch.setenv("CXXNET_FOLD_SPLIT_SUM", fold)
        trs[fold] = _net("1", monkeypatch, B)
        trs[fold].update(DataBatch(x, y))  # tunes any signature not in the table
    torch.cuda.synchronize()
    # the same weights and momentum for the compared step (the first steps' tile picks differ)
    a0, a1 = trs["0"].net.arena, trs["1"].net.arena
    a1.w.copy_(a0.w)
    a1.m1.copy_(a0.m1)
    a1.sync_shadow()
    for fold, tr in trs.items():
        w0 = {(li, s.tag): s.w.clone() for li, s in tr.net.arena.specs}
        tr.update(DataBatch(x, y))
        torch.cuda.synchronize()
        res[fold] = ({(li, s.tag): s.w - w0[(li, s.tag)] for li, s in tr.net.arena.specs},
                     sum(bool(getattr(c.layer, "folded", False)) for c in tr.net.connections))
    assert res["0"][1] == 0 and res["1"][1] >= 1, (res["0"][1], res["1"][1])
    for key, d0 in res["0"][0].items():
        d1 = res["1"][0][key]
        assert ((d1 - d0).norm() / d0.norm().clamp_min(1e-12)).item() < 5e-2, key


def _dp_worker(rank, port, steps, out):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                      CXXNET_DIST_BACKEND="nccl", CXXNET_DIST_FORCE="1")
    import torch.distributed as dist
    from cxxnet_amd.parallel import init_distributed
    init_distributed()
    tr = NetTrainer()
    base = [(k, v) for k, v in load_conf("inception_v1", []) if not k.startswith("metric")]
    for k, v in base + [("batch_size", "8"), ("dev", "gpu"), ("eval_train", "0"), ("silent", "1"), ("seed", "5"),
                        ("deterministic", "1"), ("dp_mode", "allreduce"), ("dp_bucket_mb", "4"),
                        ("cuda_graph", "0")]:
        tr.set_param(k, v)
    tr.init_model()
    assert tr.reducer.update_fn is not None and len(tr.net.sib_groups) == 9
    g = torch.Generator().manual_seed(4)
    x = torch.randn(8, 3, 224, 224, generator=g).cuda()
    y = torch.randint(0, 1000, (8, 1), generator=g).float().cuda()
    for _ in range(steps):
        tr.update(DataBatch(x, y))
    torch.cuda.synchronize()
    assert tr.reducer.check_consistency() == 0.0
    torch.save(tr.net.arena.w.cpu(), out)
    dist.destroy_process_group()


def test_inception_siblings_under_rccl_dp_match_plain(tmp_path, monkeypatch):
    """GoogLeNet with sibling groups (and folded split sums) through the data-parallel step
    (RCCL at world 1: per-bucket all-reduce from the backprop hooks -- buckets keyed by the
    groups' gradient-ready layer -- side-stream updates, forward gating) against the plain step
    of the same net, deterministic mode: the same weights after 3 steps."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "w_dp")
    mp.spawn(_dp_worker, args=(port, 3, out), nprocs=1, join=True)
    dp_w = torch.load(out, weights_only=True)
    tr = _net("1", monkeypatch, 8)
    g = torch.Generator().manual_seed(4)
    x = torch.randn(8, 3, 224, 224, generator=g).cuda()
    y = torch.randint(0, 1000, (8, 1), generator=g).float().cuda()
    for _ in range(3):
        tr.update(DataBatch(x, y))
    torch.cuda.synchronize()
    w = tr.net.arena.w.cpu()
    assert dp_w.shape == w.shape
    err = ((dp_w - w).norm() / w.norm()).item()
    assert err < 1e-5, err
