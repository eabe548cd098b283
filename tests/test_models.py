"""Model zoo: every conf builds, and one training step runs with finite results.
CPU tests cover the graph and shapes; GPU tests run the same step through the HIP
kernels and compare against the CPU executor on identical weights."""
import pytest
import torch

from cxxnet_amd.io.data import DataBatch
from cxxnet_amd.models import available, load_conf
from cxxnet_amd.nnet import NetTrainer

# (model, batch, expected output classes, input-size override for the CPU run)
ZOO = [("alexnet", 2, 1000), ("inception_v1", 2, 1000), ("vgg16", 1, 1000), ("mnist_mlp", 4, 10),
       ("mnist_conv", 4, 10), ("bowl", 4, 121)]


def _pairs(model, batch, dev, **over):
    pairs = [(k, v) for k, v in load_conf(model) if not k.startswith("metric") and k != "dev"]
    pairs += [("batch_size", str(batch)), ("eval_train", "0"), ("silent", "1"), ("dev", dev), ("seed", "3")]
    pairs = [(k, over.get(k, v)) for k, v in pairs]
    return pairs + [(k, v) for k, v in over.items() if k not in dict(pairs)]


def _trainer(pairs):
    tr = NetTrainer()
    for k, v in pairs:
        tr.set_param(k, v)
    tr.init_model()
    return tr


def _batch(tr, batch, ncls, device="cpu", seed=0):
    c, h, w = tr.net_cfg.input_shape
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(batch, c, h, w, generator=g).to(torch.bfloat16).float()
    y = torch.randint(0, ncls, (batch, 1), generator=g).float()
    return DataBatch(x.to(device), y.to(device))


def test_zoo_listed():
    assert set(m for m, _, _ in ZOO) <= set(available())


@pytest.mark.parametrize("model,batch,ncls", ZOO)
def test_model_one_step_cpu(model, batch, ncls):
    tr = _trainer(_pairs(model, batch, "cpu"))
    assert tuple(tr.net.nodes[-1].shape[1:]) == (1, 1, ncls)
    before = tr.net.arena.w.clone()
    tr.update(_batch(tr, batch, ncls))
    out = tr.net.nodes[-1].fp32_view
    assert torch.isfinite(out).all()
    assert torch.allclose(out.sum(1), torch.ones(batch), atol=1e-4)  # softmax rows
    assert torch.isfinite(tr.net.arena.w).all() and not torch.equal(before, tr.net.arena.w)


def _rel(a, b):
    a, b = a.float().cpu().reshape(-1), b.float().cpu().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.gpu
@pytest.mark.parametrize("model,batch,ncls", ZOO)
def test_model_one_step_gpu_vs_cpu(model, batch, ncls):
    # dropout off and avg pooling so both devices compute the same function
    # (bf16 vs fp32 max-pool winners legitimately differ; see test_e2e_gpu)
    over = {"threshold": "0"}
    pairs = [(k, "avg_pooling" if v == "max_pooling" else v) for k, v in _pairs(model, batch, "cpu", **over)]
    cpu = _trainer(pairs)
    gpu = _trainer([(k, "gpu" if k == "dev" else v) for k, v in pairs])
    cpu.net.arena.w.copy_(cpu.net.arena.w.to(torch.bfloat16).float())
    src = {(li, sc.tag): sc for li, sc in cpu.net.arena.specs}  # (the GPU arena may group siblings)
    for li, sg in gpu.net.arena.specs:
        sc = src[(li, sg.tag)]
        sg.w.zero_()
        sg.w[..., : sc.shape[-1]].copy_(sc.w)  # padded first-layer input channels
    gpu.net.arena.sync_shadow()
    b = _batch(cpu, batch, ncls)
    cpu.update(b)
    gpu.update(DataBatch(b.data.cuda(), b.label.cuda()))
    torch.cuda.synchronize()
    pc = cpu.net.nodes[-1].fp32_view
    pg = gpu.net.nodes[-1].fp32_view
    assert torch.isfinite(pg).all()
    assert _rel(pg, pc) < 0.05, _rel(pg, pc)
    worst = 0.0
    gsp = {(li, sg.tag): sg for li, sg in gpu.net.arena.specs}
    for li, sc in cpu.net.arena.specs:
        sg = gsp[(li, sc.tag)]
        mc = cpu.net.arena.m1[sc.offset:sc.offset + sc.numel].view(sc.shape)
        mg = gpu.net.arena.m1[sg.offset:sg.offset + sg.numel].view(sg.shape)[..., : sc.shape[-1]]
        if mc.abs().max() < 1e-12:
            continue
        worst = max(worst, _rel(mg, mc))
    assert worst < 0.15, worst
